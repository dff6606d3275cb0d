#!/bin/bash
# GPU tests, a 4-rank cyclic rehearsal on the one GPU (gloo), the cyclic per-GPU path
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -1 gpurun_out/t5.log
MOOSEX_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 4 --steps 3 --warmup 1 --size 1024 --lr-runs 0 > gpurun_out/shared4.json 2> gpurun_out/shared4.err || { tail -20 gpurun_out/shared4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/shared4.json').read().strip().splitlines()[-1]); print('shared4', d['check'], d['p2p_bytes_per_step'][0], d.get('error'))"
for s in 1 2; do
  timeout -k 10 300 python bench.py --layout cyclic --step-streams $s --steps 12 --warmup 3 --lr-runs 0 > gpurun_out/c5_$s.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/c5_$s.json').read().strip().splitlines()[-1]); print('cyc$s', round(d['ms_per_step'],2), d['check']['ok'])"
done
