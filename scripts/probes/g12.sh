set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5q}
mkdir -p $out
export MOOSEX_PARTY_STREAMS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/s0 -o run -- python scripts/probes/lr_parties_prof.py --runs 0 > $out/s0.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/s20 -o run -- python scripts/probes/lr_parties_prof.py --runs 20 > $out/s20.log 2>&1
