#!/bin/bash
# The one GPU-box runner: STEPS=<comma list> bash scripts/gpu.sh
#
# Steps (each GPU step under its own time limit; a crash, abort, fault or timeout ends the
# session at once, an assertion failure (rc 1) does not):
#   test      pytest -m gpu                      smoke     __graft_entry__ smoke()
#   driver    the driver's bench command x2 + its rocprofv3 kernel-trace summary
#   bench     bench.py, both rings              cyclic    cyclic layout on one GPU, 1/2 streams
#   shared    multi-rank rehearsal on one GPU (NS="3 8", SIZE=4096: every rank on cuda:0, gloo)
#   variants  CRT GEMM variants (VARS="8 16")    pmc       CRT GEMM PMC passes (VARS)
#   lrinf     LR-inference p50 + kernel profile dots/graphs  the dot-product sweeps
#   calls     torch calls by moose_amd call site in one eager LR inference
#   logreg    logistic-regression training sweep (LRGRAPHS=1: hipGraph replay)
#   aes       AES-in-MPC decrypt
#   coresid   GEMM + concurrent copy kernel co-residency trace
#   cycprof   rocprofv3 kernel stats of the cyclic layout's per-GPU path (one GPU)
#   ladder    the bench fallback ladder with a rank stalled in attempt 0 (one GPU, 3 ranks)
#   ab        driver command under env configurations ABCFG="name=VAR=v,VAR2=w ..." (ABPROF=1:
#             plus a rocprofv3 kernel-stats pass each)      gemmtest  the CRT GEMM GPU tests
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONPATH=$PWD TMPDIR=/tmp

run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
}

summary() {  # summary <log>: the bench line's key numbers
  python3 - "$1" <<'PY'
import json, sys
ls = [l for l in open(sys.argv[1]) if l.startswith("{")]
if not ls:
    print("no JSON line"); sys.exit(0)
d = json.loads(ls[-1])
keys = ("layout", "step_streams", "ms_per_step", "value", "check", "phase_s", "skipped",
        "attempts", "errors", "error", "lr_inference_p50_ms", "step_ms_rank0")
print({k: d[k] for k in keys if k in d})
PY
}

has() { [[ ",$STEPS," == *",$1,"* ]]; }
STEPS=${STEPS:-test,smoke,bench}

if has test; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
has smoke && run smoke 300 python __graft_entry__.py smoke
if has driver; then
  run driver1 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 && summary gpurun_out/driver1.log
  run driver2 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 && summary gpurun_out/driver2.log
  run driver_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/driver_prof -o run \
    --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
  python3 scripts/prof_summary.py gpurun_out/driver_prof/run_kernel_stats.csv \
    "driver command kernel stats" > gpurun_out/driver_prof_summary.md 2>&1 || true
fi
if has bench; then
  run bench128 600 python bench.py --steps 10 --warmup 3 && summary gpurun_out/bench128.log
  run bench64 600 python bench.py --steps 10 --warmup 3 --ring 64 && summary gpurun_out/bench64.log
fi
if has cyclic; then
  for s in 1 2; do
    run cyc_s$s 300 python bench.py --layout cyclic --steps 10 --warmup 3 --step-streams $s \
      --lr-runs 0 && summary gpurun_out/cyc_s$s.log
  done
fi
if has cycprof; then
  run cycprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cycprof -o run \
    --output-format csv -- python3 bench.py --layout cyclic --steps 10 --warmup 3 --lr-runs 0
  python3 scripts/prof_summary.py gpurun_out/cycprof/run_kernel_stats.csv \
    "cyclic layout per-GPU path (1 GPU)" > gpurun_out/cycprof_summary.md 2>&1 || true
fi
if has shared; then
  for N in ${NS:-3 8}; do
    run shared$N 600 env MOOSEX_SHARED_GPU=1 python bench.py --gpus $N --steps ${SSTEPS:-5} \
      --warmup 2 --size ${SIZE:-4096} --lr-runs 5 && summary gpurun_out/shared$N.log
  done
fi
if has ladder; then
  # the fallback ladder on a real GPU: attempt 0 (cyclic, 2 streams) hangs in its warmup on
  # rank 1, the supervisors kill it on every rank and attempt 1 (1 stream) measures
  run ladder3 400 env MOOSEX_SHARED_GPU=1 MOOSEX_BENCH_STALL=1:warmup python bench.py --gpus 3 \
    --steps 3 --warmup 1 --size 1024 --lr-runs 3 --deadline 300 && summary gpurun_out/ladder3.log
fi
if has ab; then
  # A/B of env configurations on the driver command (ABCFG="NAME=VAR=v,VAR2=w ...")
  for cfg in ${ABCFG:-base=MOOSEX_CRT_KERNEL=8}; do
    name=${cfg%%=*}; vars=${cfg#*=}
    for kv in ${vars//,/ }; do export "$kv"; done
    run ab_$name 300 python3 bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 \
      && summary gpurun_out/ab_$name.log
    if [ -n "$ABPROF" ]; then
      run abprof_$name 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_$name -o run \
        --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lr-runs 0 \
        --zero-slot-steps 0 --no-check
      python3 scripts/prof_summary.py gpurun_out/abprof_$name/run_kernel_stats.csv "$name" \
        | head -12 > gpurun_out/abprof_$name.md || true
      cat gpurun_out/abprof_$name.md
    fi
    for kv in ${vars//,/ }; do unset "${kv%%=*}"; done
  done
fi
if has gemmtest; then
  run gemmtest 600 python -u -m pytest tests/test_gemm_crt.py -m gpu -x -v --timeout 300 \
    --timeout-method thread
fi
if has variants; then
  for v in ${VARS:-8 16}; do
    run var_$v 200 env MOOSEX_CRT_KERNEL=$v python bench.py --steps 20 --warmup 5 --lr-runs 0 \
      --zero-slot-steps 0 && summary gpurun_out/var_$v.log
  done
fi
if has pmc; then
  for V in ${VARS:-8}; do
    G="python scripts/gemm_bench.py --bits 128 --iters 2 --impl crt"
    export MOOSEX_CRT_KERNEL=$V  # rocprofv3 runs the program itself: no env hop after --
    run pmc_v${V}_1 120 rocprofv3 --kernel-trace --output-format csv -o run \
      -d gpurun_out/pmc_v${V}_1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -- $G
    run pmc_v${V}_2 120 rocprofv3 --kernel-trace --output-format csv -o run \
      -d gpurun_out/pmc_v${V}_2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES \
      TCC_HIT_sum TCC_MISS_sum -- $G
    python3 scripts/pmc_summary.py gpurun_out/pmc_v${V}_1/run_counter_collection.csv \
      gpurun_out/pmc_v${V}_2/run_counter_collection.csv > gpurun_out/pmc_v${V}_summary.md 2>&1 || true
    unset MOOSEX_CRT_KERNEL
  done
fi
if has lrinf; then
  run lrinf 600 python scripts/bench_lr_inference.py --runs 50
  run lrinf_g 600 python scripts/bench_lr_inference.py --runs 50 --graphs
  run lrinf_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/lrinf_prof -o run \
    --output-format csv -- python scripts/bench_lr_inference.py --runs 5 --warmup 1
fi
if has calls; then  # torch calls by call site in one eager LR inference (the ATen copies)
  run calls 300 python scripts/probes/diag_torch_calls.py
fi
if has dots; then
  rm -f gpurun_out/dots.jsonl
  run dots 900 python benchmarks/dot_product.py --sweep --n 3 --json gpurun_out/dots.jsonl
fi
if has graphs; then
  rm -f gpurun_out/dots_graphs.jsonl
  run dots_graphs 900 python benchmarks/dot_product.py --graphs --sweep --n 3 \
    --json gpurun_out/dots_graphs.jsonl
fi
if has logreg; then
  rm -f gpurun_out/logreg.jsonl
  for it in 10 50 100; do for bs in 128 512 1024 2048; do
    run logreg_${bs}_${it} 600 python benchmarks/logreg_train.py --batch_size $bs --n_iter $it \
      --n_exp 3 --json gpurun_out/logreg.jsonl ${LRGRAPHS:+--graphs}
  done; done
fi
if has aes; then
  run aes 600 python scripts/bench_aes_decrypt.py --n 64 --runs 5
fi
if has coresid; then
  run coresid_plain 300 python3 scripts/coresidency.py --out gpurun_out/coresid_plain.json
  run coresid 300 rocprofv3 --kernel-trace --output-format csv -o run -d gpurun_out/coresid \
    -- python3 scripts/coresidency.py --out gpurun_out/coresid_traced.json
  python3 scripts/coresidency.py --summarize gpurun_out/coresid > gpurun_out/coresid_trace.json \
    2>&1 || true
fi
exit 0
