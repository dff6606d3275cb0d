#!/bin/bash
# r6: after party-batched launches -- the whole GPU suite, the 100-iteration LogReg parties
# tape (composed, merged vs not; per-party chains), smoke, and the driver's bench command
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6s
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $out/pytest.log | tail -12 | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
lr() {  # lr <name> <env...>
  local name=$1; shift
  env "$@" timeout -k 10 400 python benchmarks/logreg_train.py --runtime parties --graphs \
    --batch_size 128 --n_iter 100 --n_exp 3 > $out/logreg_$name.log 2>&1 || return $?
  echo "$name: $(grep '^{' $out/logreg_$name.log | tail -1 | cut -c1-400)"
}
lr merged || exit $?
lr unmerged MOOSEX_PARTY_MERGE=0 || exit $?
lr chains MOOSEX_PARTY_STREAMS=1 GPU_MAX_HW_QUEUES=16 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
echo "smoke rc=$?"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err
echo "bench rc=$?"
python3 -c "
import json; d=json.loads([l for l in open('$out/bench.json') if l.startswith('{')][-1])
print(d['ms_per_step'], d.get('lr_inference_p50_ms'))
lr=d.get('lr_inference',{}).get('one_gpu',{})
print({k:{kk:v.get(kk) for kk in ('p50_ms','rounds','replay_form','validated','host_issue_ms_p50')} for k,v in lr.items()})
"
