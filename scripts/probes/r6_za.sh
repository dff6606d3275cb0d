#!/bin/bash
# r6: the LogReg and dot-product tables with the parties' messages read in place
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6za
mkdir -p $out
for b in 128 512 1024 2048; do
  for it in 10 50 100; do
    timeout -k 10 400 python benchmarks/logreg_train.py --runtime parties --graphs \
      --batch_size $b --n_iter $it --n_exp 3 --json $out/logreg.jsonl > $out/lr_${b}_${it}.log 2>&1 || exit $?
    echo "$b $it $(grep '^{' $out/lr_${b}_${it}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["session_s"]["mean"],4), d["reference_s"], round(d["speedup_vs_reference"]), d["max_abs_err_vs_fp64"])')"
  done
done
timeout -k 10 900 python benchmarks/dot_product.py --runtime parties --graphs --sweep --n 5 \
  --json $out/dots.jsonl > $out/dots.log 2>&1 || exit $?
wc -l $out/dots.jsonl
