#!/bin/bash
# r6 third GPU pass: the whole GPU suite (lockstep on by default), then the "parallel" dot
# benchmark rows on per-party sessions with and without dot batching
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6c
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -12 | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for flag in 1 0; do
  for k in 10 100; do
    for n in 1 10 100; do
      MOOSEX_BATCH_DOTS=$flag timeout -k 10 240 python benchmarks/dot_product.py --runtime parties \
        --graphs --c parallel --c_arg $k --s $n --n 10 --json $out/dots_batch$flag.jsonl \
        > /dev/null 2>> $out/dots.err || exit $?
    done
  done
done
python3 -c "
import json
for f in (1, 0):
    for l in open('$out/dots_batch%d.jsonl' % f):
        d = json.loads(l)
        print('batch', f, d['k'], d['n'], round(d['seconds_median'] * 1e3, 3), 'ms ref', d['reference_s'], 'err', d['max_abs_err'])
"
