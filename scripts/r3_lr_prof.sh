#!/bin/bash
# kernel list of the LR-inference hipGraph replay (33 evaluations: 3 capture/warm + 30)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lr_prof -o run --output-format csv -- python3 scripts/r3_lr_kernels.py > gpurun_out/lr_prof.log 2>&1 || { tail -20 gpurun_out/lr_prof.log; exit 1; }
find gpurun_out/lr_prof -name "*kernel_stats.csv"
