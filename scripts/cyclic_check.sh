#!/bin/bash
# Cyclic (party-per-GPU) layout on the one-GPU box: kernel + device bitwise tests, then
# the compute cost of the per-party protocol path at N=1 with and without the row-chunked
# pipeline (exchanges are local copies at N=1), then a kernel profile.
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_cyclic.py tests/test_native_gpu.py -k "cyclic or party or rows or kp" > gpurun_out/cyclic_tests.log 2>&1 || { tail -40 gpurun_out/cyclic_tests.log; exit 1; }
tail -2 gpurun_out/cyclic_tests.log
for ch in 1 8; do
  MOOSEX_PIPELINE_CHUNKS=$ch timeout -k 10 300 python bench.py --layout cyclic --steps 5 --warmup 2 --check > gpurun_out/cyc1_ch$ch.log 2>&1 || exit $?
  tail -1 gpurun_out/cyc1_ch$ch.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chunks $ch', d['ms_per_step'], d['check'])"
done
export TMPDIR=/tmp
MOOSEX_PIPELINE_CHUNKS=${PROF_CHUNKS:-8} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cyc1_prof -o run --output-format csv -- python bench.py --layout cyclic --steps 3 --warmup 1 > gpurun_out/cyc1_prof.log 2>&1 || exit $?
echo done
