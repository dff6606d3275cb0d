#!/bin/bash
# the driver's bench command three times in a row on one box (run-to-run spread)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rep_$i.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/rep_$i.json').read().strip().splitlines()[-1])
print('run $i', round(d['ms_per_step'],3), '%.4g' % d['value'], d['step_ms_rank0'], d['check']['ok'], d['lr_inference_p50_ms'])"
done
