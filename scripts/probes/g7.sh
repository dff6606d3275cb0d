set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5l}
mkdir -p $out
timeout -k 10 300 python scripts/probes/party_streams_probe.py > $out/streams_probe.json 2> $out/streams_probe.err
