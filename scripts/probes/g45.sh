set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/${TAG:-r5az}
mkdir -p $out
for cfg in "2048 10" "128 100" "2048 100"; do
  set -- $cfg
  timeout -k 10 300 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size $1 --n_iter $2 --n_exp 5 --json $out/logreg_parties_graphs.jsonl > $out/lpg_$1_$2.log 2>&1
  rc=$?
  echo "$1 $2 rc=$rc" >> $out/rc.txt
  [ $rc -ne 0 ] && exit 0
done
exit 0
