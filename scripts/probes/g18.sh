set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5w}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/st -o run -- python bench.py --steps 10 --warmup 3 --lr-runs 0 > $out/st.log 2>&1
