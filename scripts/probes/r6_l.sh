#!/bin/bash
# r6: the composed LR / LogReg graphs' phases as the merging composer sees them
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6l
mkdir -p $out
MOOSEX_MERGE_DEBUG=1 timeout -k 10 200 python scripts/probes/graph_kernels.py --workload lr --launches 0 > $out/lr_phases.log 2>&1 || exit $?
MOOSEX_MERGE_DEBUG=1 timeout -k 10 200 python scripts/probes/graph_kernels.py --workload logreg --n_iter 2 --launches 0 > $out/logreg_phases.log 2>&1 || exit $?
grep -c "^phase" $out/lr_phases.log $out/logreg_phases.log
