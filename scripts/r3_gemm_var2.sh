#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
for cfg in ${CFGS:-"8 4" "13 4" "8 4" "13 4"}; do
  set -- $cfg
  MOOSEX_CRT_KERNEL=$1 MOOSEX_CRT_GROUPM=$2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > gpurun_out/v2_$1_$2.log 2>&1 || { tail -5 gpurun_out/v2_$1_$2.log; exit 1; }
  tail -1 gpurun_out/v2_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $1 groupm $2', round(d['ms_per_step'],2), d['step_ms_rank0']['median'], d['check']['ok'])"
done
