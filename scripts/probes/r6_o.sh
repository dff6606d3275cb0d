#!/bin/bash
# r6: where an eager per-party dot's host time goes (cProfile of party alice's thread)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6o
mkdir -p $out
EAGER_K=10 EAGER_SORT=cumulative EAGER_TOP=60 timeout -k 10 300 python scripts/probes/eager_party_prof.py > $out/eager_cum.log 2>&1 || exit $?
EAGER_K=10 EAGER_SORT=tottime EAGER_TOP=40 timeout -k 10 300 python scripts/probes/eager_party_prof.py > $out/eager_tot.log 2>&1 || exit $?
head -3 $out/eager_cum.log
