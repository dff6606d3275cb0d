#!/bin/bash
# r6: CRT GEMM tile-group height sweep under the asymmetric product (MOOSEX_CRT_GROUPM)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6grp2}
mkdir -p $out
for v in 8 4 8 4 8 4; do
  MOOSEX_CRT_GROUPM=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/b_$v.log 2>&1 || exit $?
  echo "groupm=$v $(grep -o '"ms_per_step": [0-9.]*' $out/b_$v.log)"
done
