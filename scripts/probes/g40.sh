set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5au}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_party_bits.py tests/test_threads.py -m gpu > $out/pytest.log 2>&1 &&
timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/plain.json 2> $out/plain.err &&
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 30 > $out/streams.json 2> $out/streams.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p0 -o run -- python scripts/probes/lr_parties_prof.py --runs 0 > $out/p0.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p20 -o run -- python scripts/probes/lr_parties_prof.py --runs 20 > $out/p20.log 2>&1
