#!/bin/bash
# r6: the reference's dot-product tables with the parties as separate protocol participants
# (replayed composed graphs), round-6 build
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6w
mkdir -p $out
timeout -k 10 1100 python benchmarks/dot_product.py --runtime parties --graphs --sweep --n 5 \
  --json $out/dots.jsonl > $out/dots.log 2>&1 || exit $?
wc -l $out/dots.jsonl
