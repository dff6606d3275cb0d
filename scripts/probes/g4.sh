set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5i}
mkdir -p $out
bash scripts/probes/g3.sh &&
timeout -k 10 300 python scripts/probes/party_dag_probe.py > $out/dag.json 2> $out/dag.err
