#!/bin/bash
# r6: where the one-GPU composed party replay of the LR inference spends its time
# (host issue parts, graph-only device time, kernels per replayed evaluation)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6e
mkdir -p $out
timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/lr.json 2> $out/lr.err || exit $?
cat $out/lr.json
for r in 0 20; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof$r -o run -- \
    python3 scripts/probes/lr_parties_prof.py --runs $r > $out/prof$r.log 2>&1 || exit $?
done
find $out -name "*kernel_stats.csv" | sort
