"""Host<->device argument/result paths of a graph replay (runtime/graphs.py), timed on
their own: which H2D upload and D2H read-back is cheapest for a 1000x1000 f64 argument."""
import time

import numpy as np
import torch


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return round(sorted(ts)[n // 2] * 1e3, 3)


def main():
    dev = torch.device("cuda:0")
    for n in (1000, 100):
        a = np.random.rand(n, n)
        t = torch.empty((n, n), dtype=torch.float64, device=dev)
        pin = torch.empty((n, n), dtype=torch.float64, pin_memory=True)
        res = {}
        res["to_new"] = timeit(lambda: torch.from_numpy(a).to(dev))
        res["copy_pageable"] = timeit(lambda: t.copy_(torch.from_numpy(a)))
        res["copy_pageable_nb"] = timeit(lambda: t.copy_(torch.from_numpy(a), non_blocking=True))

        def pinned():
            np.copyto(pin.numpy(), a)
            t.copy_(pin, non_blocking=True)
        res["pinned_stage"] = timeit(pinned)
        res["np_copyto_only"] = timeit(lambda: np.copyto(pin.numpy(), a))
        res["pinned_dma_only"] = timeit(lambda: t.copy_(pin, non_blocking=True))
        res["d2h_cpu"] = timeit(lambda: t.cpu().numpy())

        def d2h_pin():
            pin.copy_(t, non_blocking=True)
            torch.cuda.current_stream().synchronize()
            return pin.numpy().copy()
        res["d2h_pinned"] = timeit(d2h_pin)
        print(n, res, flush=True)


if __name__ == "__main__":
    main()
