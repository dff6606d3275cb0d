#!/bin/bash
# end-of-session check on HEAD: GPU suite, smoke, the driver's bench command, and kernel
# profiles of the driver command (stacked) and of the cyclic layout's per-GPU path
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/s2_tests.log 2>&1 || { tail -40 gpurun_out/s2_tests.log; exit 1; }
tail -1 gpurun_out/s2_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/s2_smoke.log 2>&1 || { tail -20 gpurun_out/s2_smoke.log; exit 1; }
tail -1 gpurun_out/s2_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/s2_bench.json 2> gpurun_out/s2_bench.err || { tail -20 gpurun_out/s2_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/s2_bench.json').read().strip().splitlines()[-1])
print('bench', round(d['ms_per_step'],3), d['value'], d['step_ms_rank0'], d['check']['ok'], d['lr_inference_p50_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s2_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --lr-runs 0 > gpurun_out/s2_prof.log 2>&1 || { tail -20 gpurun_out/s2_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s2_cyc -o run --output-format csv -- python3 bench.py --layout cyclic --steps 4 --warmup 1 --lr-runs 0 > gpurun_out/s2_cyc.log 2>&1 || { tail -20 gpurun_out/s2_cyc.log; exit 1; }
tail -1 gpurun_out/s2_cyc.log | cut -c1-160
find gpurun_out/s2_prof gpurun_out/s2_cyc -name "*kernel_stats.csv"
