#!/bin/bash
# r6: replay tests, LR / LogReg parties and the LogReg kernel table (messages in place)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6zc}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_storage_replay.py tests/test_merge_rounds.py \
  tests/test_batching.py tests/test_spmd.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -12 | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/lr.json 2> $out/lr.err || exit $?
cat $out/lr.json
timeout -k 10 400 python benchmarks/logreg_train.py --runtime parties --graphs \
  --batch_size 128 --n_iter 100 --n_exp 3 > $out/logreg.log 2>&1 || exit $?
grep '^{' $out/logreg.log | cut -c1-330
for n in 0 10; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof$n -o run -- \
    python3 scripts/probes/graph_kernels.py --workload logreg --launches $n > $out/prof$n.log 2>&1 || exit $?
done
grep "graph_nodes" $out/prof10.log | tail -1
python3 scripts/probes/kernel_table.py $out/prof0 $out/prof10 10 > $out/table.md
head -24 $out/table.md; tail -1 $out/table.md
