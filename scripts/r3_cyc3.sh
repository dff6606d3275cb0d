#!/bin/bash
# GPU tests, then the cyclic per-GPU path with 1 / 2 / 3 step streams (8 HW queues) vs stacked
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -40 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --lr-runs 0 > gpurun_out/c3_stacked.json 2> gpurun_out/c3_stacked.err || exit 1
for s in 1 2 3; do
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --layout cyclic --step-streams $s --steps 12 --warmup 3 --lr-runs 0 > gpurun_out/c3_cyc$s.json 2> gpurun_out/c3_cyc$s.err || exit 1
done
python3 - <<'PY'
import json
for f in ("stacked", "cyc1", "cyc2", "cyc3"):
    d = json.loads(open(f"gpurun_out/c3_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 2), d.get("check", {}).get("ok"))
PY
