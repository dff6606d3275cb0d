#!/bin/bash
# CRT GEMM: GPU tests (both kernel variants), GEMM timing (CRT vs limb), headline bench.
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gemm_crt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/crt_tests.log 2>&1 || { tail -30 gpurun_out/crt_tests.log; exit 1; }
tail -2 gpurun_out/crt_tests.log
MOOSEX_CRT_KERNEL=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_crt.py -x -q --timeout 120 --timeout-method thread -k gpu > gpurun_out/crt_tests_k1.log 2>&1 || { tail -30 gpurun_out/crt_tests_k1.log; exit 1; }
tail -1 gpurun_out/crt_tests_k1.log
for k in 1 2; do
  MOOSEX_CRT_KERNEL=$k timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 128 --iters 5 --impl crt 2>&1 | grep -v amdgpu.ids
  MOOSEX_CRT_KERNEL=$k timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 64 --iters 5 --impl crt 2>&1 | grep -v amdgpu.ids
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --check 2>&1 | tail -1
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --check --ring 64 2>&1 | tail -1
