#!/bin/bash
# Parallel-dots batching and the hipGraph replay at 1000^2: kernel profile of the batched
# k=100 case, and graph replay timing alone vs after a sweep.
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/dot_product.py --c parallel --s 1000 --c_arg 100 --n 3 > gpurun_out/par100.log 2>&1 || exit $?
tail -1 gpurun_out/par100.log
MOOSEX_BATCH_DOTS=0 timeout -k 10 300 python benchmarks/dot_product.py --c parallel --s 1000 --c_arg 100 --n 3 > gpurun_out/par100_nobatch.log 2>&1 || exit $?
tail -1 gpurun_out/par100_nobatch.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/par100_prof -o run --output-format csv -- python benchmarks/dot_product.py --c parallel --s 1000 --c_arg 100 --n 1 > gpurun_out/par100_prof.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/dot_product.py --graphs --c seq --s 1000 --c_arg 1 --n 5 > gpurun_out/g1000.log 2>&1 || exit $?
tail -1 gpurun_out/g1000.log
timeout -k 10 300 python -c "
import sys; sys.argv=['x','--graphs','--sweep','--n','3']
sys.path.insert(0,'benchmarks')
import dot_product as dp
dp.main(['--graphs','--c','seq','--s','100','--c_arg','100','--n','3'])
dp.main(['--graphs','--c','seq','--s','1000','--c_arg','1','--n','5'])
dp.main(['--c','seq','--s','1000','--c_arg','1','--n','5'])
" > gpurun_out/gsweep.log 2>&1 || exit $?
cat gpurun_out/gsweep.log | grep '^{'
