set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5p}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_threads.py -m gpu > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
timeout -k 10 300 python scripts/probes/party_dag_probe.py > $out/dag_pool_landing.json 2> $out/dag1.err
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/party_dag_probe.py > $out/dag_persistent_landing.json 2> $out/dag2.err
