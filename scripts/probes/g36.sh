set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5aq}
mkdir -p $out
timeout -k 10 200 python scripts/probes/eager_party_prof.py > $out/eager.log 2>&1
