#!/bin/bash
# r6: the cyclic per-GPU path's kernel table under the asymmetric products
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6cyc}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --layout cyclic --steps 10 --warmup 2 --lr-runs 0 --zero-slot-steps 0 > $out/prof.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*' $out/prof.log
python3 scripts/probes/db_table.py $out/prof 12
