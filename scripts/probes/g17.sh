set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5v}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "cyclic" > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
timeout -k 10 300 python bench.py --layout cyclic --steps 20 --warmup 5 --lr-runs 0 > $out/c1.json 2> $out/c1.err &&
MOOSEX_DEALER_SIDE=0 timeout -k 10 300 python bench.py --layout cyclic --steps 20 --warmup 5 --lr-runs 0 > $out/c0.json 2> $out/c0.err &&
timeout -k 10 300 python bench.py --layout cyclic --steps 20 --warmup 5 --lr-runs 0 > $out/c2.json 2> $out/c2.err
