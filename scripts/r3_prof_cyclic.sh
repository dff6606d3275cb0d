#!/bin/bash
# kernel profile of the cyclic layout's per-GPU path at N=1 (exchanges are device copies)
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cyc_prof -o run --output-format csv -- python3 bench.py --layout cyclic --steps 4 --warmup 1 --lr-runs 0 --no-check ${EXTRA} > gpurun_out/cyc_prof.log 2>&1 || { tail -20 gpurun_out/cyc_prof.log; exit 1; }
tail -1 gpurun_out/cyc_prof.log
