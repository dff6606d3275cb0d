#!/bin/bash
# round 3, GPU pass B: per-party dot tail on the device, cyclic bitwise test, cyclic N=1 timing
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_party_tail.py tests/test_cyclic.py tests/test_native_gpu.py -k "party or cyclic or tail" > gpurun_out/b_tests.log 2>&1 || { tail -30 gpurun_out/b_tests.log; exit 1; }
tail -2 gpurun_out/b_tests.log
for s in 1 2; do
  timeout -k 10 300 python bench.py --layout cyclic --steps 10 --warmup 3 --step-streams $s --lr-runs 0 > gpurun_out/b_cyc_s$s.log 2>&1 || { tail -20 gpurun_out/b_cyc_s$s.log; exit 1; }
  tail -1 gpurun_out/b_cyc_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cyclic streams $s', d['ms_per_step'], d['check'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cyc_prof2 -o run --output-format csv -- python3 bench.py --layout cyclic --steps 4 --warmup 1 --lr-runs 0 --no-check > gpurun_out/cyc_prof2.log 2>&1 || { tail -20 gpurun_out/cyc_prof2.log; exit 1; }
