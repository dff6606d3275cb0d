set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/${TAG:-r5bf}
mkdir -p $out
export MOOSEX_PARTY_GRAPH_FLAT=all
for rep in 1 2; do
for cfg in "128 10" "2048 10" "128 100" "2048 100"; do
  set -- $cfg
  timeout -k 10 300 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size $1 --n_iter $2 --n_exp 5 --json $out/logreg_all.jsonl > $out/lpg_$1_$2_$rep.log 2>&1
  rc=$?
  echo "$rep $1 $2 rc=$rc" >> $out/rc.txt
  [ $rc -ne 0 ] && exit 0
done
done
timeout -k 10 600 python -X faulthandler benchmarks/dot_product.py --runtime parties --graphs --sweep --n 5 --json $out/dots_all.jsonl > $out/dg.log 2>&1
echo "dots rc=$?" >> $out/rc.txt
exit 0
