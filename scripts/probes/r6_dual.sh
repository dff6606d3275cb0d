#!/bin/bash
# r6: share image and its sum from one read (MOOSEX_CRT_DUAL) -- A/B
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6dual}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_dot_asym.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -4 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 1 0 1 0; do
  MOOSEX_CRT_DUAL=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/b_$v.log 2>&1 || exit $?
  echo "dual=$v $(grep -o '"ms_per_step": [0-9.]*' $out/b_$v.log)"
done
for v in 1 0; do
  MOOSEX_CRT_DUAL=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof$v -o run -- python3 bench.py --steps 10 --warmup 2 --lr-runs 0 --zero-slot-steps 0 > $out/prof$v.log 2>&1 || exit $?
  python3 scripts/probes/db_table.py $out/prof$v 12 | head -10
done
