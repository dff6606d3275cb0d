set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5af}
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/plain$i.json 2> $out/plain$i.err || exit 1
  MOOSEX_PARTY_STREAMS=1 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/streams$i.json 2> $out/streams$i.err || exit 1
  MOOSEX_PARTY_STREAMS=1 MOOSEX_PARTY_LAUNCH_THREADS=0 timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/streams_nothr$i.json 2> $out/streams_nothr$i.err || exit 1
done
