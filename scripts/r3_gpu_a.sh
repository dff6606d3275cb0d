#!/bin/bash
# round 3, GPU pass A: new GPU tests, the default bench line (matmul + check + LR p50),
# the cyclic layout at N=1 with 1 and 2 step streams.
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_lanes.py > gpurun_out/a_tests.log 2>&1 || { tail -30 gpurun_out/a_tests.log; exit 1; }
tail -2 gpurun_out/a_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/a_bench.log 2>&1 || { tail -20 gpurun_out/a_bench.log; exit 1; }
tail -1 gpurun_out/a_bench.log
for s in 1 2; do
  timeout -k 10 300 python bench.py --layout cyclic --steps 10 --warmup 3 --step-streams $s --lr-runs 0 > gpurun_out/a_cyc_s$s.log 2>&1 || { tail -20 gpurun_out/a_cyc_s$s.log; exit 1; }
  tail -1 gpurun_out/a_cyc_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cyclic streams $s', d['ms_per_step'], d['check'])"
done
