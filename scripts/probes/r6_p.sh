#!/bin/bash
# r6: eager per-party dots (seq k = 100 at n = 1) under the round-6 interpreter flags
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6p
mkdir -p $out
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python benchmarks/dot_product.py --runtime parties --c seq --c_arg 100 --s 1 \
    --n 3 > $out/$name.json 2>> $out/err.log || return $?
  echo "$name $(python3 -c "import json; d=json.loads(open('$out/$name.json').read().splitlines()[-1]); print(round(d['seconds_mean']*1e3,1))")"
}
run default || exit $?
run nolockstep MOOSEX_LOCKSTEP=0 || exit $?
run nobatch MOOSEX_BATCH_DOTS=0 || exit $?
run noscopes MOOSEX_NONCE_SCOPES=0 || exit $?
run nomerge MOOSEX_MERGE_ROUNDS=0 || exit $?
run none MOOSEX_LOCKSTEP=0 MOOSEX_BATCH_DOTS=0 MOOSEX_MERGE_ROUNDS=0 || exit $?
