#!/bin/bash
# One GPU-box session: tests, smoke, headline bench (both rings), kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" \
&& timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
&& timeout -k 10 600 python bench.py --steps 5 --warmup 2 --check > gpurun_out/bench128.log 2>&1 && cat gpurun_out/bench128.log \
&& timeout -k 10 600 python bench.py --steps 5 --warmup 2 --ring 64 --check > gpurun_out/bench64.log 2>&1 && cat gpurun_out/bench64.log \
&& cd /tmp && export TMPDIR=/tmp && cd - >/dev/null \
&& timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 && echo "prof ok"
