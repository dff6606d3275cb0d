set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/${TAG:-r5ba}
mkdir -p $out
MOOSEX_FLAT_DEBUG=1 timeout -k 10 300 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size 2048 --n_iter 10 --n_exp 2 > $out/lpg.log 2>&1
echo "rc=$?" >> $out/rc.txt
grep -v "^flat: " $out/lpg.log > $out/lpg_nodbg.log || true
tail -c 3000 $out/lpg.log > $out/lpg_tail.log
grep -c "^flat: " $out/lpg.log >> $out/rc.txt || true
rm -f $out/lpg.log
exit 0
