"""Calibration: the library (hipBLASLt via torch._int_mm) int8 GEMM rate on this GPU at the
shape of one CRT-GEMM slice of the headline bench (M=N=4096, K'=8192), random operands."""
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    for (m, k, n) in ((4096, 8192, 4096), (8192, 8192, 8192)):
        a = torch.randint(-128, 128, (m, k), dtype=torch.int8, device=dev)
        b = torch.randint(-128, 128, (k, n), dtype=torch.int8, device=dev)
        try:
            for _ in range(3):
                torch._int_mm(a, b)
            torch.cuda.synchronize()
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                torch._int_mm(a, b)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            print(f"_int_mm {m}x{k}x{n}: {dt*1e3:.3f} ms  {2*m*n*k/dt/1e15:.2f} POPS", flush=True)
        except Exception as e:  # noqa: BLE001
            print("_int_mm failed:", e, flush=True)
        try:
            af = a.to(torch.float8_e4m3fn)
            bf = b.to(torch.float8_e4m3fn).t().contiguous().t()
            one = torch.ones((), device=dev)
            for _ in range(3):
                torch._scaled_mm(af, bf, one, one, out_dtype=torch.bfloat16)
            torch.cuda.synchronize()
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                torch._scaled_mm(af, bf, one, one, out_dtype=torch.bfloat16)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            print(f"fp8 scaled_mm {m}x{k}x{n}: {dt*1e3:.3f} ms  {2*m*n*k/dt/1e15:.2f} PFLOPS",
                  flush=True)
        except Exception as e:  # noqa: BLE001
            print("scaled_mm failed:", e, flush=True)


if __name__ == "__main__":
    main()
