"""Time the stacked RSS cross GEMM (the Dot hot kernel) alone: 3 x (M x 2K) . (2K x N)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from moose_amd.ops import ring as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--bits", type=int, default=128)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--peak", action="store_true", help="also run the MFMA peak probe")
    ap.add_argument("--impl", default="both", choices=["crt", "limb", "both"])
    ap.add_argument("--sweep", action="store_true",
                    help="sweep the tile-order knobs (MOOSEX_GEMM_GROUPM / MOOSEX_GEMM_XCD)")
    a = ap.parse_args()
    if a.peak:
        mfma_peak()
    n, bits = a.n, a.bits
    shp = (3, n, n) + ((2,) if bits == 128 else ())
    g = torch.Generator(device="cuda").manual_seed(0)
    xs = [R.RT(torch.randint(-2**62, 2**62, shp, device="cuda", generator=g), bits) for _ in range(4)]
    from moose_amd.ops import native as nat

    L = 16 if bits == 128 else 8
    for impl in (("crt", "limb") if a.impl == "both" else (a.impl,)):
        nat.lib().mx_set_gemm_crt(1 if impl == "crt" else 2)
        nmul = nat.lib().mx_crt_moduli(bits // 64, 2 * n) if impl == "crt" else L * (L + 1) // 2
        R.dot_cross(*xs, nb=1)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            R.dot_cross(*xs, nb=1)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        ops = 2 * 3 * n * n * 2 * n * nmul
        print(f"n={n} bits={bits} {impl} ({nmul} int8 GEMMs per party): {dt*1e3:.2f} ms/call  "
              f"{ops/dt/1e15:.2f} int8 POPS executed", flush=True)
    nat.lib().mx_set_gemm_crt(0)
    if a.sweep:
        import os

        for xcd in ("1", "0"):
            for gm in ("1", "2", "4", "8", "16"):
                os.environ["MOOSEX_GEMM_GROUPM"], os.environ["MOOSEX_GEMM_XCD"] = gm, xcd
                R.dot_cross(*xs, nb=1)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(a.iters):
                    R.dot_cross(*xs, nb=1)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) / a.iters
                print(f"  xcd={xcd} group_m={gm}: {dt*1e3:.2f} ms/call "
                      f"{ops/dt/1e15:.2f} int8 POPS", flush=True)



def mfma_peak(blocks=1024, iters=20000):
    """Register-only v_mfma_i32_32x32x32_i8 rate (the ceiling for the limb GEMM)."""
    from moose_amd.ops import native as nat

    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    nat.lib().mx_mfma_peak(blocks, 10, nat.ptr(sink), st)
    torch.cuda.synchronize()
    t = time.perf_counter()
    nat.lib().mx_mfma_peak(blocks, iters, nat.ptr(sink), st)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ops = blocks * 4 * iters * 8 * 2 * 32 * 32 * 32
    print(f"mfma peak probe: {ops / dt / 1e15:.2f} int8 POPS ({blocks} blocks x 4 waves)")


if __name__ == "__main__":
    main()
