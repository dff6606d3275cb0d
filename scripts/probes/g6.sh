set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5k}
mkdir -p $out
timeout -k 10 300 python scripts/probes/party_mem_probe.py > $out/mem.json 2> $out/mem.err
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_party_bits.py tests/test_party_jobs.py tests/test_native_gpu.py tests/test_graphs.py tests/test_spmd.py tests/test_keys.py -m gpu > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
