#!/bin/bash
# r6: composed replays with a fourth (outsider) party -- receiving an output, owning an
# input (replayable fresh seeds) -- and the SPMD/party suites around them
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6u
mkdir -p $out
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py tests/test_spmd.py tests/test_storage_replay.py tests/test_merge_rounds.py \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|^E " $out/pytest.log | head -20 | cut -c1-300
