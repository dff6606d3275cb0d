#!/bin/bash
# r6: the headline step's kernels alone (no LR inference, no zero-slot extra): steps 10 minus
# steps 0 of the same command, per step
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6n
mkdir -p $out
for s in 2 12; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d $out/prof$s -o run -- \
    python3 bench.py --steps $s --warmup 1 --lr-runs 0 --zero-slot-steps 0 > $out/bench$s.log 2>&1 || exit $?
done
grep '^{' $out/bench12.log | cut -c1-200
python3 scripts/probes/kernel_table.py $out/prof2 $out/prof12 10 > $out/table.md
cat $out/table.md
