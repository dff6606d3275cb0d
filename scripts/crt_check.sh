cd /root/repo && mkdir -p gpurun_out && export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gemm_crt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/crt_tests.log 2>&1; rc=$?; tail -5 gpurun_out/crt_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 128 --iters 5 2>&1 | tee gpurun_out/crt_gemm128.log
timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 64 --iters 5 2>&1 | tee gpurun_out/crt_gemm64.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --check 2>&1 | tail -1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --check --ring 64 2>&1 | tail -1
