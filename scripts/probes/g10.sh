set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5o}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_threads.py -m gpu > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
timeout -k 10 300 python scripts/probes/party_streams_probe.py > $out/streams_probe.json 2> $out/streams_probe.err
timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 20 > $out/plain.json 2> $out/plain.err &&
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 20 > $out/streams.json 2> $out/streams.err
