#!/bin/bash
# full GPU suite + smoke + driver bench command, then the 4-wave 128x128 GEMM variants
# (12-15, built with the VGPR-form MFMA flag) against the default 8 on the same box
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/full_bench.log 2>&1 || { tail -20 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log
for v in ${VARS:-8 12 13 14 15 8 12}; do
  MOOSEX_CRT_KERNEL=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > gpurun_out/v12_$v.log 2>&1 || { tail -5 gpurun_out/v12_$v.log; exit 1; }
  tail -1 gpurun_out/v12_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $v', round(d['ms_per_step'],2), d['step_ms_rank0'], d['check']['ok'])"
done
