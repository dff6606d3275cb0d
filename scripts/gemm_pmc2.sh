#!/bin/bash
# LDS / MFMA counters of the limb GEMM (kernel-trace + pmc only).
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc3 -o run --output-format csv -- python scripts/gemm_bench.py --bits 128 --iters 2 > gpurun_out/pmc3.log 2>&1 || exit $?
MOOSEX_GEMM_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/pmc4 -o run --output-format csv -- python scripts/gemm_bench.py --bits 128 --iters 2 > gpurun_out/pmc4.log 2>&1 || exit $?
echo done
