#!/bin/bash
# persistent CRT GEMM (variant 15): bit-exact tests, then timing against variant 8
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_crt.py -m gpu -k "persistent or bench_tiling" > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
CFGS="8 4|15 4|8 4|15 4" 
IFS='|'; for cfg in $CFGS; do
  IFS=' '; set -- $cfg
  MOOSEX_CRT_KERNEL=$1 MOOSEX_CRT_GROUPM=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 > gpurun_out/e_$1.log 2>&1 || { tail -5 gpurun_out/e_$1.log; exit 1; }
  tail -1 gpurun_out/e_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $1', round(d['ms_per_step'],2), d['check']['ok'])"
done
