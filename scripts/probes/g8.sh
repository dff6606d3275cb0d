set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5m}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_threads.py -m gpu -k "device_flag" > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
