#!/bin/bash
# r6 second GPU pass: the whole GPU suite, smoke, then the driver's bench command
cd "$(dirname "$0")/../.."
export PYTHONPATH=$PWD TMPDIR=/tmp
out=gpurun_out/r6b
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests \
  > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 $out/pytest.log | cut -c1-300
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
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
