set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5n}
mkdir -p $out
timeout -k 10 120 python -X faulthandler -u scripts/probes/flag_probe.py > $out/flag.log 2>&1
echo "rc=$?" >> $out/flag.log
