set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5ak}
mkdir -p $out
MOOSEX_GRAPHS_DEBUG=1 timeout -k 10 200 python -u benchmarks/dot_product.py --runtime parties --graphs --c seq --s 1000 --c_arg 1 --n 3 > $out/d1000.log 2>&1
MOOSEX_GRAPHS_DEBUG=1 timeout -k 10 200 python -u benchmarks/dot_product.py --runtime parties --graphs --c seq --s 100 --c_arg 1 --n 3 > $out/d100.log 2>&1
exit 0
