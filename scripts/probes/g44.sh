set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ay}
mkdir -p $out
MOOSEX_PARTY_GRAPH_FLAT=0 timeout -k 10 200 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size 2048 --n_iter 10 --n_exp 2 > $out/child.log 2>&1
echo "child rc=$?" >> $out/rc.txt
MOOSEX_PARTY_GRAPH_FLAT=1 timeout -k 10 200 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size 2048 --n_iter 10 --n_exp 2 > $out/flat.log 2>&1
echo "flat rc=$?" >> $out/rc.txt
exit 0
