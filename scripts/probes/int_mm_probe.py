"""How fast is the vendor int8 GEMM (torch._int_mm -> hipBLASLt) on the CRT GEMM's shape,
4096 x 8192 x 4096 int8 -> int32, compared with k_crt_gemm16 (108 of them in 10.8 ms)?"""
import time

import torch


def main():
    dev = torch.device("cuda:0")
    a = torch.randint(-127, 127, (4096, 8192), dtype=torch.int8, device=dev)
    b = torch.randint(-127, 127, (8192, 4096), dtype=torch.int8, device=dev)
    bt = b.t().contiguous().t()  # column-major B
    for name, bb in (("row-major B", b), ("col-major B", bt)):
        try:
            for _ in range(3):
                torch._int_mm(a, bb)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            n = 20
            for _ in range(n):
                torch._int_mm(a, bb)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / n
            ops = 2 * 4096 * 8192 * 4096
            print(f"{name}: {dt * 1e3:.3f} ms per GEMM, {ops / dt / 1e15:.2f} POPS; "
                  f"108 GEMMs: {108 * dt * 1e3:.1f} ms (+ a mod-p pass over 7.2 GB of int32)",
                  flush=True)
        except Exception as e:  # noqa: BLE001
            print(name, "failed:", e)


if __name__ == "__main__":
    main()
