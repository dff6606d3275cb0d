#!/bin/bash
# cyclic layout at N=1 (1 and 2 step streams) vs stacked, then a kernel profile of cyclic
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --lr-runs 0 > gpurun_out/cn_stacked.json 2> gpurun_out/cn_stacked.err || exit 1
for s in 1 2; do
  timeout -k 10 300 python bench.py --layout cyclic --step-streams $s --steps 10 --warmup 3 --lr-runs 0 > gpurun_out/cn_cyc$s.json 2> gpurun_out/cn_cyc$s.err || exit 1
done
python3 - <<'PY'
import json
for f in ("stacked", "cyc1", "cyc2"):
    d = json.loads(open(f"gpurun_out/cn_{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"], 2), d.get("step_ms_rank0"), d.get("check"))
PY
bash scripts/r3_prof_cyclic.sh
