set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5t}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_threads.py tests/test_merge_rounds.py -m gpu > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/streams.json 2> $out/streams.err &&
MOOSEX_PARTY_STREAMS=1 MOOSEX_PARTY_LAUNCH_THREADS=0 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/streams_nothreads.json 2> $out/streams_nothreads.err &&
timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/plain.json 2> $out/plain.err
