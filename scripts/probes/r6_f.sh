#!/bin/bash
# r6: party-batched launches in the composed one-GPU replay -- the replay tests, then the LR
# inference replay's host issue / device time / dispatches (as r6_e.sh)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6f
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_storage_replay.py tests/test_merge_rounds.py \
  tests/test_batching.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -12 | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/lr.json 2> $out/lr.err || exit $?
MOOSEX_PARTY_MERGE=0 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/lr_nomerge.json 2>> $out/lr.err || exit $?
cat $out/lr.json $out/lr_nomerge.json
for r in 0 20; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof$r -o run -- \
    python3 scripts/probes/lr_parties_prof.py --runs $r > $out/prof$r.log 2>&1 || exit $?
done
