#!/bin/bash
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6_queue
mkdir -p $out
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace -d $out/q$q -o run --output-format csv \
    -- python3 scripts/probes/queue_probe.py 6 > $out/q$q.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob
for q in (4, 16):
    f = glob.glob(f"gpurun_out/r6_queue/q{q}/**/run_kernel_trace.csv", recursive=True) or \
        glob.glob(f"gpurun_out/r6_queue/q{q}/run_kernel_trace.csv")
    rows = list(csv.DictReader(open(f[0])))
    print("GPU_MAX_HW_QUEUES", q, [(r["Grid_Size_X"], r["Queue_Id"], r["Stream_Id"]) for r in rows if "Fill" in r["Kernel_Name"]])
PY
