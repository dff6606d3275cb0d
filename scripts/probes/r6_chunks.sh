#!/bin/bash
# r6: row-chunked stacked dot pipeline (MOOSEX_STACKED_CHUNKS) -- headline step time per T,
# then one kernel trace at T=4 (overlap of the tails with the GEMM chunks)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6_chunks
mkdir -p $out
for T in 1 2 4 8; do
  MOOSEX_STACKED_CHUNKS=$T timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 \
    > $out/t$T.json 2> $out/t$T.err || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('$out/t$T.json') if l.startswith('{')][-1]); print('T=$T', d['ms_per_step'], d.get('check'), d.get('step_ms_rank0'))"
done
MOOSEX_STACKED_CHUNKS=${TRACE_T:-4} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run \
  --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lr-runs 0 > $out/prof.log 2>&1
