#!/bin/bash
# r6: composed replay with a fourth (outsider) party: why the tape capture declines
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6u
mkdir -p $out
MOOSEX_GRAPHS_DEBUG=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_threads.py -k "outsider" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "Error|error|^E " $out/pytest.log | head -30 | cut -c1-300
