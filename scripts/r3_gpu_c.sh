#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gemm_crt.py -m gpu > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c_bench.log 2>&1 || { tail -5 gpurun_out/c_bench.log; exit 1; }
tail -1 gpurun_out/c_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', round(d['ms_per_step'],2), d['step_ms_rank0'], d['check'], d['lr_inference_p50_ms'])"
MOOSEX_CRT_KERNEL=6 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --lr-runs 0 > gpurun_out/c_bench6.log 2>&1 || { tail -5 gpurun_out/c_bench6.log; exit 1; }
tail -1 gpurun_out/c_bench6.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench v6', round(d['ms_per_step'],2))"
