#!/bin/bash
# hipGraph replay vs eager on the reference dot sweep rows where replay lost in round 2,
# forced replay (PROBES=0) and adaptive; then a kernel trace of eager vs replayed steps
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/g_*.jsonl
for c in "seq 1 1000" "parallel 1 1000" "seq 10 1000" "parallel 10 100" "seq 1 1"; do
  set -- $c
  timeout -k 10 300 python benchmarks/dot_product.py --c $1 --c_arg $2 --s $3 --n 20 --json gpurun_out/g_eager.jsonl > /dev/null 2>&1 || exit 1
  MOOSEX_GRAPHS_PROBES=0 timeout -k 10 300 python benchmarks/dot_product.py --graphs --c $1 --c_arg $2 --s $3 --n 20 --json gpurun_out/g_forced.jsonl > /dev/null 2>&1 || exit 1
  timeout -k 10 300 python benchmarks/dot_product.py --graphs --c $1 --c_arg $2 --s $3 --n 20 --json gpurun_out/g_adaptive.jsonl > /dev/null 2>&1 || exit 1
done
python - <<'PY'
import json
rows = {}
for mode in ("eager", "forced", "adaptive"):
    for l in open(f"gpurun_out/g_{mode}.jsonl"):
        d = json.loads(l); rows.setdefault((d["mode"], d["k"], d["n"]), {})[mode] = d["seconds_median"] * 1e3
for k, v in rows.items():
    print(k, {m: round(x, 3) for m, x in v.items()})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g_prof_eager -o run --output-format csv -- python3 benchmarks/dot_product.py --c seq --c_arg 1 --s 1000 --n 5 > /dev/null 2>&1 || exit 1
MOOSEX_GRAPHS_PROBES=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g_prof_graph -o run --output-format csv -- python3 benchmarks/dot_product.py --graphs --c seq --c_arg 1 --s 1000 --n 5 > /dev/null 2>&1 || exit 1
echo done
