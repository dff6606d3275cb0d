set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ax}
mkdir -p $out
timeout -k 10 600 python -u benchmarks/dot_product.py --runtime parties --graphs --sweep --n 5 --json $out/dots_parties_graphs.jsonl > $out/dg.log 2>&1 || exit 1
for cfg in "128 10" "2048 10" "128 100" "2048 100"; do
  set -- $cfg
  timeout -k 10 300 python benchmarks/logreg_train.py --runtime parties --graphs --batch_size $1 --n_iter $2 --n_exp 5 --json $out/logreg_parties_graphs.jsonl > $out/lpg_$1_$2.log 2>&1 || exit 1
done
