#!/bin/bash
# repeated four-rank rehearsals of the cyclic layout on one GPU (gloo staging): the output
# check of every run (a staged receive raced its host buffer before the pinned fix)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for i in ${RUNS:-1 2 3 4 5 6}; do
  MOOSEX_BENCH_RUN_DIR=$PWD/gpurun_out/r4_$i MOOSEX_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 4 --steps 3 --warmup 1 --size 1024 --lr-runs 3 --watchdog 100 > gpurun_out/r4_$i.json 2> gpurun_out/r4_$i.err
  echo "run $i rc=$?"
  python3 -c "
import json; d=json.loads(open('gpurun_out/r4_$i.json').read().strip().splitlines()[-1])
print(d['check'], d.get('error'), d.get('errors'))"
done
