#!/bin/bash
# CRT GEMM variant 16 (one barrier per two k-steps, five stage buffers): bit-exactness at
# the bench tiling, then the driver's bench step against the default 8 on the same box
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_crt.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v16_tests.log 2>&1 || { tail -30 gpurun_out/v16_tests.log; exit 1; }
tail -1 gpurun_out/v16_tests.log
for v in ${VARS:-8 16 8 16 8 16}; do
  MOOSEX_CRT_KERNEL=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > gpurun_out/v16_$v.log 2>&1 || { tail -5 gpurun_out/v16_$v.log; exit 1; }
  tail -1 gpurun_out/v16_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $v', round(d['ms_per_step'],3), d['step_ms_rank0'], d['check']['ok'])"
done
