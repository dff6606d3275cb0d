#!/bin/bash
# r6: messages read in place (threads.Mailbox): replay tests, then LR and LogReg parties
# with and without it
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6z}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_storage_replay.py tests/test_merge_rounds.py \
  tests/test_batching.py tests/test_spmd.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -12 | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for ip in 1 0; do
  MOOSEX_PARTY_INPLACE=$ip timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 \
    > $out/lr$ip.json 2> $out/lr$ip.err || exit $?
  echo "inplace=$ip"; cat $out/lr$ip.json
  MOOSEX_PARTY_INPLACE=$ip timeout -k 10 400 python benchmarks/logreg_train.py --runtime parties \
    --graphs --batch_size 128 --n_iter 100 --n_exp 3 > $out/logreg$ip.log 2>&1 || exit $?
  grep '^{' $out/logreg$ip.log | cut -c1-400
done
