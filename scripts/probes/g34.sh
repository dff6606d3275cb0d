set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ao}
mkdir -p $out
for i in 1 2 3; do
  MOOSEX_JOBS_FOLD=1 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/fold$i.json 2> $out/fold$i.err || exit 1
  MOOSEX_JOBS_FOLD=0 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/nofold$i.json 2> $out/nofold$i.err || exit 1
done
