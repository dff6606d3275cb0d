#!/bin/bash
# r6: the reference's dot-product tables, parties as separate participants, EAGER (every
# evaluation interpreted: what a first evaluation pays), round-6 build with the baton
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6y2
mkdir -p $out
timeout -k 10 1100 python benchmarks/dot_product.py --runtime parties --sweep --n 3 \
  --json $out/dots_eager.jsonl > $out/dots.log 2>&1 || exit $?
wc -l $out/dots_eager.jsonl
