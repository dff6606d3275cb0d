#!/bin/bash
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
for P in 1 0 1 0; do
  MOOSEX_KEYS_PINNED=$P timeout -k 10 120 python scripts/bench_lr_inference.py --runs 100 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pinned $P eager p50', round(d['value'],3), 'p90', round(d['p90_ms'],3))"
done
