set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5u}
mkdir -p $out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 > $out/b1.json 2> $out/b1.err &&
MOOSEX_BENCH_STREAMS=2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 > $out/b2.json 2> $out/b2.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 > $out/b3.json 2> $out/b3.err
