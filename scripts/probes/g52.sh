set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/${TAG:-r5bg}
mkdir -p $out
MOOSEX_PARTY_GRAPH_FLAT=all MOOSEX_FLAT_DEBUG=1 timeout -k 10 300 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size 128 --n_iter 100 --n_exp 2 > $out/dbg.log 2>&1
echo "dbg rc=$?" >> $out/rc.txt
grep -v "^flat: " $out/dbg.log | grep -v "Extension" | tail -12 >> $out/rc.txt || true
grep -c "^flat: " $out/dbg.log >> $out/rc.txt || true
grep "^flat: " $out/dbg.log | tail -2 >> $out/rc.txt || true
rm -f $out/dbg.log
exit 0
