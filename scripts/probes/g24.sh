set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ad}
mkdir -p $out
timeout -k 10 300 python bench.py --layout cyclic --lr-runs 0 --zero-slot-steps 0 > $out/cyc.json 2> $out/cyc.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/pc -o run -- python bench.py --layout cyclic --lr-runs 0 --zero-slot-steps 0 --steps 10 > $out/pc.log 2>&1
