"""Do kernels on different PyTorch streams run concurrently on this device, given the HIP
hardware-queue count (GPU_MAX_HW_QUEUES)?  For every pair (long GEMM on stream i, short
kernel on stream j issued right after) the short kernel's completion time is compared with
the GEMM's: 'overlap' when it finishes long before the GEMM does.  bench.py's cyclic layout
relies on this: one step's RCCL kernels (on the communicator's stream) must run while the
next step's GEMM occupies the CUs."""
import json
import os
import sys
import time

import torch


def main():
    dev = torch.device("cuda:0")
    nstreams = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    kind = sys.argv[2] if len(sys.argv) > 2 else "rocblas"
    if kind == "crt":  # the bench's own CRT GEMM: 27648 workgroups, one resident per CU
        sys.path.insert(0, os.getcwd())
        from moose_amd.ops import ring as R

        n = 4096
        g = torch.Generator(device=dev).manual_seed(0)
        mk = lambda: R.RT(torch.randint(-2**62, 2**62, (3, n, n, 2), device=dev,  # noqa: E731
                                        dtype=torch.int64, generator=g), 128)
        x0, x1, y0, y1 = mk(), mk(), mk(), mk()
        reps = 1

        def long_op():
            R.dot_cross(x0, x1, y0, y1, nb=1)
    else:
        a = torch.randn(8192, 8192, device=dev, dtype=torch.float32)
        b = torch.randn(8192, 8192, device=dev, dtype=torch.float32)
        reps = 4

        def long_op():
            a @ b
    small = torch.zeros(1 << 16, device=dev)
    torch.cuda.synchronize()
    # warm up both kernels on every stream
    for s in streams:
        with torch.cuda.stream(s):
            long_op()
            small.add_(1)
    torch.cuda.synchronize()
    res = {}
    for i in range(nstreams):
        for j in range(nstreams):
            if i == j:
                continue
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            torch.cuda.synchronize()
            with torch.cuda.stream(streams[i]):
                e0.record()
                for _ in range(reps):
                    long_op()
                e1.record()
            with torch.cuda.stream(streams[j]):
                small.add_(1)
                e2.record()
            torch.cuda.synchronize()
            gemm = e0.elapsed_time(e1)
            short = e0.elapsed_time(e2)
            res[f"{i}->{j}"] = round(short / gemm, 3)
    over = sum(1 for v in res.values() if v < 0.5)
    print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "long": kind,
                      "streams": nstreams, "pairs_overlapping": over, "pairs": len(res),
                      "ratio_short_done_over_gemm": res}), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
