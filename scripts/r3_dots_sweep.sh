#!/bin/bash
# the reference dot-product sweep (BASELINE tables), eager and hipGraph replay (default mode)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/sw_eager.jsonl gpurun_out/sw_graphs.jsonl
timeout -k 10 400 python benchmarks/dot_product.py --sweep --n 9 --json gpurun_out/sw_eager.jsonl > gpurun_out/sw_eager.log 2>&1 || { tail -20 gpurun_out/sw_eager.log; exit 1; }
timeout -k 10 400 python benchmarks/dot_product.py --sweep --graphs --n 9 --json gpurun_out/sw_graphs.jsonl > gpurun_out/sw_graphs.log 2>&1 || { tail -20 gpurun_out/sw_graphs.log; exit 1; }
python3 - <<'PY'
import json
rows = {}
for mode in ("eager", "graphs"):
    for l in open(f"gpurun_out/sw_{mode}.jsonl"):
        d = json.loads(l)
        rows.setdefault((d["mode"], d["k"], d["n"]), {})[mode] = d["seconds_median"] * 1e3
worse = 0
for k, v in rows.items():
    flag = "" if v["graphs"] <= v["eager"] else "  <-- graphs slower"
    worse += bool(flag)
    print(k, {m: round(x, 3) for m, x in v.items()}, flag)
print("rows where graphs > eager:", worse)
PY
