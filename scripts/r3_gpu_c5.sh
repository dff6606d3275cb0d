#!/bin/bash
# one-GPU rehearsal of the N >= 3 / N >= 6 bench paths (ranks share the GPU, gloo staging):
# cyclic headline + LR SPMD + configs 2/3 (+ config 5 at six ranks)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for N in ${NS:-3 6}; do
  MOOSEX_BENCH_RUN_DIR=$PWD/gpurun_out/run$N MOOSEX_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus $N --steps 3 --warmup 1 --size 1024 --lr-runs 3 > gpurun_out/shared$N.json 2> gpurun_out/shared$N.err || { grep -v "Gloo\|hostname" gpurun_out/shared$N.err | tail -30; cat gpurun_out/run$N/*.json; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/shared$N.json').read().strip().splitlines()[-1])
print('shared$N', d['layout'], round(d['ms_per_step'],2), d['check'], d.get('errors'))
print('lr', d.get('lr_inference_p50_ms'))
print('c23', d.get('spmd_three_gpus'))
print('c5', d.get('config5_dp2_replicas'))"
done
