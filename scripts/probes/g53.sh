set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/${TAG:-r5bh}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_threads.py tests/test_party_bits.py -m gpu > $out/pytest.log 2>&1 || exit 1
timeout -k 10 200 python scripts/probes/lr_parties_prof.py --runs 50 > $out/plain.json 2> $out/plain.err || exit 1
for cfg in "128 10" "2048 10" "128 100" "2048 100"; do
  set -- $cfg
  timeout -k 10 300 python -X faulthandler benchmarks/logreg_train.py --runtime parties --graphs --batch_size $1 --n_iter $2 --n_exp 5 --json $out/logreg.jsonl > $out/lpg_$1_$2.log 2>&1
  rc=$?
  echo "$1 $2 rc=$rc" >> $out/rc.txt
  [ $rc -ne 0 ] && exit 0
done
timeout -k 10 600 python -X faulthandler benchmarks/dot_product.py --runtime parties --graphs --sweep --n 5 --json $out/dots.jsonl > $out/dg.log 2>&1
echo "dots rc=$?" >> $out/rc.txt
exit 0
