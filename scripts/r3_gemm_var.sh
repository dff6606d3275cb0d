#!/bin/bash
# CRT GEMM variants: gemm_bench timing + full bench per MOOSEX_CRT_KERNEL value
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for V in ${VARIANTS:-6 7}; do
  export MOOSEX_CRT_KERNEL=$V
  timeout -k 10 200 python scripts/gemm_bench.py --bits 128 --impl crt --iters 10 2>&1 | grep POPS || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 > gpurun_out/var_$V.log 2>&1 || { tail -5 gpurun_out/var_$V.log; exit 1; }
  tail -1 gpurun_out/var_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $V bench', round(d['ms_per_step'],2), d['check']['ok'])"
done
