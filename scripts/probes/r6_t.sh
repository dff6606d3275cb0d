#!/bin/bash
# r6: kernels of one replayed stacked LR inference (runs 20 minus runs 0)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6t
mkdir -p $out
for r in 0 20; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof$r -o run -- \
    python3 scripts/probes/lr_parties_prof.py --mode stacked --runs $r > $out/prof$r.log 2>&1 || exit $?
done
grep '^{' $out/prof20.log | cut -c1-300
python3 scripts/probes/kernel_table.py $out/prof0 $out/prof20 20 > $out/table.md
cat $out/table.md
