#!/bin/bash
# r6: eager per-party evaluations with and without the baton (one party's Python at a
# time), then the party/thread GPU tests
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6x2
mkdir -p $out
for b in 1 1; do
  for k in 1 100; do
    MOOSEX_PARTY_BATON=$b timeout -k 10 300 python benchmarks/dot_product.py --runtime parties --c seq \
      --c_arg $k --s 1 --n 5 > $out/d_${b}_${k}.json 2>> $out/err.log || exit $?
    echo "baton=$b seq k=$k: $(python3 -c "import json; d=json.loads(open('$out/d_${b}_${k}.json').read().splitlines()[-1]); print(round(d['seconds_mean']*1e3,2), 'ms')")"
  done
done
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_merge_rounds.py tests/test_batching.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -5 | cut -c1-300
