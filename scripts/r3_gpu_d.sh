#!/bin/bash
# LR eager A/B (pinned key writes), PMC of the default GEMM variant 8, cyclic N=1 timing
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r3_lr_ab.sh || exit 1
VARIANTS="8" bash scripts/r3_gemm_pmc.sh > gpurun_out/pmc8.log 2>&1 || { tail -5 gpurun_out/pmc8.log; exit 1; }
grep -E "effective clock|MFMA pipe|WAIT_ANY/|WAIT_INST_ANY/|L2 hit|mean dispatch" gpurun_out/pmc_v8_summary.md | grep gemm16 | cut -c 90-
for s in 1 2; do
  timeout -k 10 300 python bench.py --layout cyclic --steps 10 --warmup 3 --step-streams $s --lr-runs 0 > gpurun_out/d_cyc_s$s.log 2>&1 || { tail -20 gpurun_out/d_cyc_s$s.log; exit 1; }
  tail -1 gpurun_out/d_cyc_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cyclic streams $s', d['ms_per_step'], d['check']['ok'])"
done
