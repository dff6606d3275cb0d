#!/bin/bash
# PMC counters of the limb GEMM, one rocprofv3 pass per counter group (kernel-trace + pmc
# only), plus a plain timing run.  Usage: BITS=128 TAG=v0 scripts/gemm_pmc.sh
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
BITS=${BITS:-128}
TAG=${TAG:-cur}
O=gpurun_out/pmc_${TAG}_${BITS}
timeout -k 10 300 python scripts/gemm_bench.py --bits $BITS --peak --impl ${IMPL:-both} > ${O}_time.log 2>&1 || exit $?
cat ${O}_time.log
P="timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -o run"
G="python scripts/gemm_bench.py --bits $BITS --iters 2 --impl ${IMPL:-both}"
$P -d ${O}_1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT -- $G > ${O}_1.log 2>&1 || exit $?
$P -d ${O}_2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES TCC_HIT_sum TCC_MISS_sum -- $G > ${O}_2.log 2>&1 || exit $?
python scripts/pmc_summary.py ${O}_1/run_counter_collection.csv ${O}_2/run_counter_collection.csv > ${O}_summary.md 2>&1
cat ${O}_summary.md
echo done
