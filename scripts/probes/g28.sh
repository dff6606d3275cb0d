set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ai}
mkdir -p $out
for cfg in "128 10" "2048 10" "128 100" "2048 100"; do
  set -- $cfg
  timeout -k 10 240 python benchmarks/logreg_train.py --runtime parties --batch_size $1 --n_iter $2 --n_exp 5 --json $out/logreg_parties.jsonl > $out/lp_$1_$2.log 2>&1 || exit 1
  echo "eager $1 $2 done" >> $out/progress.txt
  timeout -k 10 300 python benchmarks/logreg_train.py --runtime parties --graphs --batch_size $1 --n_iter $2 --n_exp 5 --json $out/logreg_parties_graphs.jsonl > $out/lpg_$1_$2.log 2>&1 || exit 1
  echo "graphs $1 $2 done" >> $out/progress.txt
done
