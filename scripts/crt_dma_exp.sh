cd /root/repo && export PYTHONPATH=$PWD
for m in 3 1 0; do for k in 1 2; do
echo "mask=$m kernel=$k"; MOOSEX_CRT_DMA_MASK=$m MOOSEX_CRT_KERNEL=$k timeout -k 10 200 python scripts/gemm_bench.py --n 4096 --bits 128 --iters 3 --impl crt 2>&1 | grep -v amdgpu.ids
done; done
