#!/bin/bash
# PMC counters of the limb GEMM (each pass in its own rocprofv3 run, kernel-trace only).
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
BITS=${BITS:-128}
timeout -k 10 300 python scripts/gemm_bench.py --bits $BITS > gpurun_out/gemm_bench_$BITS.log 2>&1 || exit $?
cat gpurun_out/gemm_bench_$BITS.log
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA -d gpurun_out/pmc1_$BITS -o run --output-format csv -- python scripts/gemm_bench.py --bits $BITS --iters 2 > gpurun_out/pmc1_$BITS.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc2_$BITS -o run --output-format csv -- python scripts/gemm_bench.py --bits $BITS --iters 2 > gpurun_out/pmc2_$BITS.log 2>&1 || exit $?
echo done
