#!/bin/bash
# r6: segment flattening without the round-5 caps.  Copy / memset nodes
# are never flattened (their read-back parameters are garbage on this runtime: the round-5
# crash); kernel-only segments are, with no 200-segment executables and no 256-segment cap.
# The 100-iteration LogReg parties tape (benchmarks/logreg_train.py, batch 128):
#   composed_nocap  ONE composed executable, every kernel-only segment flattened
#   chain_nocap     per-party stream graphs (mx_graph_build_chain), the same flattening
#   old_default     round-5 defaults (200-segment executables, 256-segment cap)
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
ulimit -c 0
out=gpurun_out/r6_flat3
mkdir -p $out
run() {  # run <name> <env...>
  local name=$1; shift
  env "$@" MOOSEX_FLAT_DEBUG=1 timeout -k 10 400 python benchmarks/logreg_train.py \
    --runtime parties --graphs --batch_size 128 --n_iter 100 --n_exp 3 > $out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc flat nodes: $(grep -c '^flat: node' $out/$name.log)"
  sed -i '/^flat: /d' $out/$name.log
  grep -v Extension $out/$name.log | grep "compose:\|MIN/MAX\|^[0-9]\|fault\|Error" | tail -6 | cut -c1-300
  return $rc
}
run composed_nocap MOOSEX_PARTY_GRAPH_CHUNK=100000 MOOSEX_FLAT_MAX_SEGMENTS=0 || exit $?
run chain_nocap MOOSEX_PARTY_STREAMS=1 GPU_MAX_HW_QUEUES=16 MOOSEX_FLAT_MAX_SEGMENTS=0 || exit $?
run old_default || exit $?
