#!/bin/bash
# full GPU test suite + smoke + the driver's bench command
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
tail -1 gpurun_out/full_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/full_bench.log 2>&1 || { tail -20 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log
