set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5aa}
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
for i in 1 2 3; do timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/plain$i.json 2> $out/plain$i.err || break; done
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/streams.json 2> $out/streams.err
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err
