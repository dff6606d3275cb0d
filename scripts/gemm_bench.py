"""Time the stacked RSS cross GEMM (the Dot hot kernel) alone: 3 x (M x 2K) . (2K x N)."""
import argparse
import time

import torch

from moose_amd.ops import ring as R


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    n, bits = a.n, a.bits
    shp = (3, n, n) + ((2,) if bits == 128 else ())
    g = torch.Generator(device="cuda").manual_seed(0)
    xs = [R.RT(torch.randint(-2**62, 2**62, shp, device="cuda", generator=g), bits) for _ in range(4)]
    R.dot_cross(*xs, nb=1)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        R.dot_cross(*xs, nb=1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.iters
    L = 16 if bits == 128 else 8
    ops = 2 * 3 * n * n * 2 * n * L * (L + 1) / 2
    print(f"n={n} bits={bits} {dt*1e3:.2f} ms/call  {ops/dt/1e15:.2f} int8 POPS")


if __name__ == "__main__":
    main()
