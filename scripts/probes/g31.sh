set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5al}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_threads.py -m gpu > $out/pytest.log 2>&1 &&
timeout -k 10 700 python -u benchmarks/dot_product.py --runtime parties --graphs --sweep --n 5 --json $out/dots_parties_graphs.jsonl > $out/dg.log 2>&1 &&
timeout -k 10 500 python -u benchmarks/dot_product.py --runtime parties --sweep --n 3 --json $out/dots_parties.jsonl > $out/de.log 2>&1
