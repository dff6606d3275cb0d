set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ac}
mkdir -p $out
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/party_dag_probe.py --reps 2 > $out/dag_persist.json 2> $out/dag_persist.err
