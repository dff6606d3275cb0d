#!/bin/bash
# r6 first GPU pass: queue mapping, the changed GPU tests, the chunked-pipeline probe
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r6a
bash scripts/probes/r6_queue.sh > gpurun_out/r6a/queue.txt 2>&1; echo "queue rc=$?"
tail -4 gpurun_out/r6a/queue.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_reveal_precision.py tests/test_party_bits.py tests/test_storage_replay.py \
  > gpurun_out/r6a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r6a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/probes/r6_chunks.sh
