set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r5j}
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_keys.py tests/test_threads.py tests/test_party_jobs.py tests/test_native_gpu.py tests/test_spmd.py tests/test_party_tail.py tests/test_party_bits.py tests/test_graphs.py -m gpu > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/pytest.log
timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 20 > $out/plain.json 2> $out/plain.err &&
MOOSEX_PARTY_STREAMS=1 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 20 > $out/streams.json 2> $out/streams.err
MOOSEX_PARTY_STREAMS=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python scripts/probes/lr_parties_prof.py --runs 20 > $out/streams8.json 2> $out/streams8.err
timeout -k 10 300 python scripts/probes/party_dag_probe.py > $out/dag.json 2> $out/dag.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p0 -o run -- python scripts/probes/lr_parties_prof.py --runs 0 > $out/p0.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/p20 -o run -- python scripts/probes/lr_parties_prof.py --runs 20 > $out/p20.log 2>&1
