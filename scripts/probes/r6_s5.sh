#!/bin/bash
# r6: full GPU suite, smoke, driver bench, and per-party large dots (asymmetric per-party products)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6s5}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -8 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || exit $?
grep '^{' $out/bench.log > $out/bench_line.json; cut -c1-200 $out/bench_line.json
for a in 1 0; do
  for s in 1000 512; do
    MOOSEX_DOT_ASYM=$a timeout -k 10 300 python benchmarks/dot_product.py --runtime parties --graphs --c seq --s $s --c_arg 1 --n 5 > $out/dots_${a}_$s.log 2>&1 || exit $?
    echo "parties dot asym=$a n=$s: $(grep '^{' $out/dots_${a}_$s.log | cut -c1-250)"
  done
done
