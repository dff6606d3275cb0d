#!/bin/bash
# r6: full GPU suite, smoke, the driver's bench and the cyclic per-GPU path (asym vs sym)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6s3}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -8 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || exit $?
grep '^{' $out/bench.log > $out/bench_line.json; cut -c1-300 $out/bench_line.json
for a in 1 0; do
  MOOSEX_DOT_ASYM=$a timeout -k 10 300 python bench.py --layout cyclic --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/cyc_$a.log 2>&1 || exit $?
  echo "cyclic asym=$a $(grep -o '"ms_per_step": [0-9.]*' $out/cyc_$a.log)"
done
