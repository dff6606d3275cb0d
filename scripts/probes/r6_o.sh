#!/bin/bash
# r6: where an eager per-party dot's host time goes (cProfile of party alice's thread)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6o
mkdir -p $out
EAGER_K=1 EAGER_SORT=tottime EAGER_TOP=45 timeout -k 10 300 python scripts/probes/eager_party_prof.py > $out/eager_k1.log 2>&1 || exit $?
head -3 $out/eager_k1.log
