set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ar}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_party_bits.py -m gpu > $out/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  MOOSEX_WSUM_GROUP=1 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/g$i.json 2> $out/g$i.err || exit 1
  MOOSEX_WSUM_GROUP=0 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/t$i.json 2> $out/t$i.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p0 -o run -- python scripts/probes/lr_parties_prof.py --runs 0 > $out/p0.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p20 -o run -- python scripts/probes/lr_parties_prof.py --runs 20 > $out/p20.log 2>&1
