set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/${TAG:-r5bd}
mkdir -p $out
MOOSEX_PARTY_GRAPH_FLAT=all MOOSEX_FLAT_DEBUG=1 timeout -k 10 300 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size 2048 --n_iter 10 --n_exp 2 > $out/dbg.log 2>&1
echo "dbg rc=$?" >> $out/rc.txt
grep "^flat: " $out/dbg.log | tail -5 >> $out/rc.txt || true
grep "^flat: " $out/dbg.log | awk '{print $7, $9}' | sort | uniq -c | sort -rn | head -20 >> $out/rc.txt || true
rm -f $out/dbg.log
exit 0
