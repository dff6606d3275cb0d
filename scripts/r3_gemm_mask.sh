#!/bin/bash
# what the CRT GEMM's data movement costs: MOOSEX_CRT_DMA_MASK (wrong results; timing only)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
for M in 3 0 1 2 11 8; do
  MOOSEX_CRT_DMA_MASK=$M timeout -k 10 200 python scripts/gemm_bench.py --bits 128 --impl crt --iters 10 2>&1 | grep POPS | sed "s/^/mask $M: /" || exit 1
done
