#!/bin/bash
# CRT GEMM: GPU tests for every kernel variant, GEMM timing per variant, headline bench.
cd "$(dirname "$0")/.." && mkdir -p gpurun_out && export PYTHONPATH=$PWD
for k in 5 6; do
  MOOSEX_CRT_KERNEL=$k timeout -k 10 300 python -u -m pytest tests/test_gemm_crt.py -x -q --timeout 120 --timeout-method thread -k gpu > gpurun_out/crt_tests_k$k.log 2>&1 || { tail -30 gpurun_out/crt_tests_k$k.log; exit 1; }
  echo "kernel $k: $(tail -1 gpurun_out/crt_tests_k$k.log)"
done
for k in 5 6; do
  MOOSEX_CRT_KERNEL=$k timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 128 --iters 5 --impl crt 2>&1 | grep -v amdgpu.ids
  MOOSEX_CRT_KERNEL=$k timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 64 --iters 5 --impl crt 2>&1 | grep -v amdgpu.ids
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --check 2>&1 | tail -1 | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --check --ring 64 2>&1 | tail -1 | cut -c1-200
