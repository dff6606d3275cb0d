#!/bin/bash
# One GPU-box session: tests, smoke, headline bench (both rings), kernel profile.
# A step that fails an assertion (rc 1) does not stop the session; a crash, abort,
# fault or timeout (any other non-zero rc) ends it immediately.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONPATH=$PWD

run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
}

STEPS=${STEPS:-all}
if [[ $STEPS == *driver* ]]; then
  # the driver's exact bench command, twice, then under rocprofv3 (kernel trace only)
  (rocm-smi --showclocks --showpower --showperflevel > gpurun_out/smi_before.txt 2>&1 || true)
  run driver1 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  run driver2 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
  run default 300 python3 bench.py
  (rocm-smi --showclocks --showpower --showperflevel > gpurun_out/smi_after.txt 2>&1 || true)
  export TMPDIR=/tmp
  run driver_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/driver_prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5
fi
[[ $STEPS == *test* || $STEPS == all ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
[[ $STEPS == *smoke* || $STEPS == all ]] && run smoke 300 python __graft_entry__.py smoke
[[ $STEPS == *bench* || $STEPS == all ]] && run bench128 600 python bench.py --steps 5 --warmup 2 --check
[[ $STEPS == *bench* || $STEPS == all ]] && run bench64 600 python bench.py --steps 5 --warmup 2 --ring 64 --check
if [[ $STEPS == *multi* || $STEPS == all ]]; then
  # multi-rank layouts rehearsed on the one GPU (ranks share cuda:0, payloads via gloo)
  export MOOSEX_SHARED_GPU=1
  run cyclic3 600 python bench.py --gpus 3 --layout cyclic --size 1024 --steps 3 --warmup 1 --check
  run spmd3 600 python bench.py --gpus 3 --layout spmd --size 1024 --steps 3 --warmup 1 --check
  unset MOOSEX_SHARED_GPU
fi
if [[ $STEPS == *aes* ]]; then
  run aes_bp 600 python scripts/bench_aes_decrypt.py --n 64 --runs 5
  MOOSEX_AES_SBOX=algebraic run aes_alg 600 python scripts/bench_aes_decrypt.py --n 64 --runs 3
fi
if [[ $STEPS == *logreg* ]]; then
  rm -f gpurun_out/logreg.jsonl
  for it in 10 50 100; do for bs in 128 512 1024 2048; do
    run logreg_${bs}_${it} 600 python benchmarks/logreg_train.py --batch_size $bs --n_iter $it --n_exp 3 --json gpurun_out/logreg.jsonl
  done; done
fi
if [[ $STEPS == *dots* ]]; then
  rm -f gpurun_out/dots.jsonl
  run dots 900 python benchmarks/dot_product.py --sweep --n 3 --json gpurun_out/dots.jsonl
fi
if [[ $STEPS == *graphs* ]]; then
  run pytest_graphs 600 python -m pytest tests/test_graphs.py tests/test_keys.py -x -q
  rm -f gpurun_out/logreg_graphs.jsonl gpurun_out/dots_graphs.jsonl
  for it in 10 100; do for bs in 128 2048; do
    run logreg_g_${bs}_${it} 900 python benchmarks/logreg_train.py --graphs --batch_size $bs --n_iter $it --n_exp 3 --json gpurun_out/logreg_graphs.jsonl
  done; done
  run dots_graphs 900 python benchmarks/dot_product.py --graphs --sweep --n 3 --json gpurun_out/dots_graphs.jsonl
fi
if [[ $STEPS == *quick* ]]; then
  rm -f gpurun_out/logreg_quick.jsonl
  run lq_e_128_10 600 python benchmarks/logreg_train.py --batch_size 128 --n_iter 10 --n_exp 3 --json gpurun_out/logreg_quick.jsonl
  run lq_e_128_100 600 python benchmarks/logreg_train.py --batch_size 128 --n_iter 100 --n_exp 2 --json gpurun_out/logreg_quick.jsonl
  run lq_g_128_100 600 python benchmarks/logreg_train.py --graphs --batch_size 128 --n_iter 100 --n_exp 3 --json gpurun_out/logreg_quick.jsonl
  run lq_g_2048_100 600 python benchmarks/logreg_train.py --graphs --batch_size 2048 --n_iter 100 --n_exp 3 --json gpurun_out/logreg_quick.jsonl
fi
if [[ $STEPS == *lrinf* ]]; then
  run lrinf128 600 python scripts/bench_lr_inference.py --runs 50
  run lrinf64 600 python scripts/bench_lr_inference.py --runs 50 --ring 64
  run lrinf128g 600 python scripts/bench_lr_inference.py --runs 50 --graphs
  run lrinf64g 600 python scripts/bench_lr_inference.py --runs 50 --ring 64 --graphs
  export TMPDIR=/tmp
  run lrinf_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/lrinf_prof -o run --output-format csv -- python scripts/bench_lr_inference.py --runs 5 --warmup 1
fi
if [[ $STEPS == *prof* || $STEPS == all ]]; then
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1
  run prof64 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --ring 64
fi
exit 0
