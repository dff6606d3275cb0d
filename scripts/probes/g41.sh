set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5av}
mkdir -p $out
timeout -k 10 200 python -u -m pytest -x -v -W always --timeout 120 --timeout-method thread "tests/test_threads.py::test_thread_party_tapes_replay_bitwise_equal_eager" -m gpu > $out/pytest.log 2>&1
AMD_LOG_LEVEL=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_threads.py::test_thread_party_tapes_replay_bitwise_equal_eager[streams]" -m gpu > $out/pytest_log2.log 2>&1
exit 0
