#!/bin/bash
# r6: packed residues on the B' prep (MOOSEX_CRT_PACKED_B) -- A/B, then the full GPU suite
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6pkb}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_dot_asym.py tests/test_gemm_crt.py > $out/pytest_crt.log 2>&1
rc=$?; echo "pytest(crt) rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest_crt.log | tail -3 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
MOOSEX_CRT_PACKED_B=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_dot_asym.py tests/test_gemm_crt.py > $out/pytest_pkb.log 2>&1
rc=$?; echo "pytest(packed B) rc=$rc"; tail -1 $out/pytest_pkb.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 1 0 1 0; do
  MOOSEX_CRT_PACKED_B=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/b_$v.log 2>&1 || exit $?
  echo "packed_b=$v $(grep -o '"ms_per_step": [0-9.]*' $out/b_$v.log)"
done
for v in 1 0; do
  MOOSEX_CRT_PACKED_B=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof$v -o run -- python3 bench.py --steps 10 --warmup 2 --lr-runs 0 --zero-slot-steps 0 > $out/prof$v.log 2>&1 || exit $?
  python3 scripts/probes/db_table.py $out/prof$v 12 | grep prep
done
