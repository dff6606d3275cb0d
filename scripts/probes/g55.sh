set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5bj}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_threads.py tests/test_party_bits.py -m gpu > $out/pytest.log 2>&1 &&
timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 30 > $out/plain.json 2> $out/plain.err
