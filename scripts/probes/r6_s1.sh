#!/bin/bash
# r6 re-entry: full GPU suite, smoke and a short bench on the rebuilt tree
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6s1}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -8 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1 || exit $?
tail -1 $out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || exit $?
grep '^{' $out/bench.log | cut -c1-400
