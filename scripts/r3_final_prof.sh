#!/bin/bash
# kernel profile of the driver's bench command (stacked, one GPU) + the noisy sweep row again
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --lr-runs 0 > gpurun_out/fin_prof.log 2>&1 || { tail -20 gpurun_out/fin_prof.log; exit 1; }
tail -1 gpurun_out/fin_prof.log | cut -c1-200
rm -f gpurun_out/row_*.jsonl
for i in 1 2; do
  timeout -k 10 120 python benchmarks/dot_product.py --c parallel --c_arg 1 --s 10 --n 21 --json gpurun_out/row_eager.jsonl > /dev/null 2>&1 || exit 1
  timeout -k 10 120 python benchmarks/dot_product.py --graphs --c parallel --c_arg 1 --s 10 --n 21 --json gpurun_out/row_graphs.jsonl > /dev/null 2>&1 || exit 1
done
python3 - <<'PY'
import json
for m in ("eager", "graphs"):
    for l in open(f"gpurun_out/row_{m}.jsonl"):
        d = json.loads(l)
        print(m, round(d["seconds_median"] * 1e3, 3), [round(x * 1e3, 3) for x in d["seconds_all"]])
PY
