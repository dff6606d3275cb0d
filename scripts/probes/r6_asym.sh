#!/bin/bash
# r6: asymmetric local products (five K-long GEMMs instead of six) -- tests, A/B bench, kernel table
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/${OUT:-r6asym3}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_dot_asym.py tests/test_gemm_crt.py > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -8 | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/bench_asym.log 2>&1 || exit $?
grep '^{' $out/bench_asym.log | cut -c1-330
MOOSEX_DOT_ASYM=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lr-runs 0 --zero-slot-steps 0 > $out/bench_sym.log 2>&1 || exit $?
grep '^{' $out/bench_sym.log | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --lr-runs 0 --zero-slot-steps 0 > $out/prof.log 2>&1 || exit $?
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {} | cut -c1-200'
