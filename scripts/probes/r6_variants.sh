#!/bin/bash
# r6: CRT GEMM variant sweep under the asymmetric product (MOOSEX_CRT_KERNEL)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6var}
mkdir -p $out
for v in 8 9 10 11 16 6 8; do
  MOOSEX_CRT_KERNEL=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/b_$v.log 2>&1 || exit $?
  echo "variant=$v $(grep -o '"ms_per_step": [0-9.]*' $out/b_$v.log)"
done
