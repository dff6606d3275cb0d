#!/bin/bash
# r6: one-GPU party replay forms -- composed total order (default), composed DAG
# (MOOSEX_PARTY_GRAPH_DAG=1), per-party stream graphs (own hardware queues) -- on the LR
# inference (p50) and the 100-iteration LogReg training; then the new GPU tests
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6_dag
mkdir -p $out
for cfg in "total" "dag MOOSEX_PARTY_GRAPH_DAG=1" "streams MOOSEX_PARTY_STREAMS=1 GPU_MAX_HW_QUEUES=16"; do
  set -- $cfg; name=$1; shift
  env "$@" timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 30 > $out/lr_$name.json 2> $out/lr_$name.err || exit $?
  echo "lr $name: $(tail -1 $out/lr_$name.json | cut -c1-400)"
  env "$@" timeout -k 10 300 python benchmarks/logreg_train.py --runtime parties --graphs \
    --batch_size 128 --n_iter 100 --n_exp 3 > $out/logreg_$name.log 2>&1 || exit $?
  echo "logreg $name: $(grep -A1 MIN/MAX $out/logreg_$name.log | tail -1)"
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_storage_replay.py tests/test_party_kernels_gpu.py \
  > $out/pytest.log 2>&1
echo "pytest rc=$?"; tail -4 $out/pytest.log
