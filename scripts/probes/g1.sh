set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5a
timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 20 > gpurun_out/r5a/plain.json 2> gpurun_out/r5a/plain.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a/p0 -o run -- python scripts/probes/lr_parties_prof.py --runs 0 > gpurun_out/r5a/p0.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r5a/p20 -o run -- python scripts/probes/lr_parties_prof.py --runs 20 > gpurun_out/r5a/p20.log 2>&1
