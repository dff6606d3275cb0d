#!/bin/bash
# GEMM kernel iteration on the GPU box: exactness tests, then timing of both kernel
# generations (v2 default, MOOSEX_GEMM_V=1 = round-1 kernels) and the bench step.
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_native_gpu.py -k "gemm" > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -3 gpurun_out/gemm_tests.log
for bits in 128 64; do
  timeout -k 10 200 python scripts/gemm_bench.py --bits $bits > gpurun_out/gemm_v2_$bits.log 2>&1 || exit $?
  cat gpurun_out/gemm_v2_$bits.log
  MOOSEX_GEMM_V=1 timeout -k 10 200 python scripts/gemm_bench.py --bits $bits > gpurun_out/gemm_v1_$bits.log 2>&1 || exit $?
  cat gpurun_out/gemm_v1_$bits.log
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --check > gpurun_out/bench128.log 2>&1 || exit $?
tail -1 gpurun_out/bench128.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --ring 64 --check > gpurun_out/bench64.log 2>&1 || exit $?
tail -1 gpurun_out/bench64.log
