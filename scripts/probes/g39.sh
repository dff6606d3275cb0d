set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5at}
mkdir -p $out
MOOSEX_PARTY_GRAPH_FLAT=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_threads.py tests/test_party_bits.py -m gpu > $out/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  MOOSEX_PARTY_GRAPH_FLAT=1 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/flat$i.json 2> $out/flat$i.err || exit 1
  MOOSEX_PARTY_GRAPH_FLAT=0 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/child$i.json 2> $out/child$i.err || exit 1
done
