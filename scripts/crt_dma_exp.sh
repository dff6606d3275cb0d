#!/bin/bash
# Attribution experiments for the CRT GEMM (timing only; results are wrong by design).
cd "$(dirname "$0")/.." && export PYTHONPATH=$PWD
for k in 1 2; do for m in 3 7 11 0 4 8 12; do
echo "kernel=$k mask=$m"; MOOSEX_CRT_DMA_MASK=$m MOOSEX_CRT_KERNEL=$k timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 128 --iters 3 --impl crt 2>&1 | grep -v amdgpu.ids
done; done
