#!/bin/bash
# r6: kernels of one composed per-party LogReg training replay (10 iterations, batch 128):
# which launches stay single per party (graph-only launches, scripts/probes/graph_kernels.py)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6h
mkdir -p $out
for n in 0 10; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof$n -o run -- \
    python3 scripts/probes/graph_kernels.py --workload logreg --launches $n > $out/prof$n.log 2>&1 || exit $?
done
tail -1 $out/prof10.log
python3 scripts/probes/kernel_table.py $out/prof0 $out/prof10 10 > $out/table.md
head -50 $out/table.md
