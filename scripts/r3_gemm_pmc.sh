#!/bin/bash
# CRT GEMM PMC passes for the given variants (MOOSEX_CRT_KERNEL), one rocprofv3 run per pass
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for V in ${VARIANTS:-6}; do
  export MOOSEX_CRT_KERNEL=$V
  O=gpurun_out/pmc_v${V}
  timeout -k 10 200 python scripts/gemm_bench.py --bits 128 --impl crt --iters 5 > ${O}_time.log 2>&1 || exit $?
  cat ${O}_time.log
  G="python scripts/gemm_bench.py --bits 128 --iters 2 --impl crt"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -o run -d ${O}_1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT -- $G > ${O}_1.log 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -o run -d ${O}_2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum -- $G > ${O}_2.log 2>&1 || exit $?
  python scripts/pmc_summary.py ${O}_1/run_counter_collection.csv ${O}_2/run_counter_collection.csv > ${O}_summary.md 2>&1
  grep -v "prep\|recon" ${O}_summary.md | grep gemm | cut -c 80- 
done
