set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5r}
mkdir -p $out
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/party_dag_probe.py > $out/dag.json 2> $out/dag.err
