"""Do kernels on different HIP streams overlap -- eagerly and inside a replayed hipGraph
with parallel branches?  Each branch is a chain of short spin kernels
(torch.cuda._sleep); prints wall time for 1 branch and for B branches on B streams."""
import time

import torch


def chain(n, cycles):
    for _ in range(n):
        torch.cuda._sleep(cycles)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    n, cycles = 50, 20000
    for branches in (1, 2, 4):
        streams = [torch.cuda.Stream() for _ in range(branches)]
        main_s = torch.cuda.current_stream()

        def eager():
            ev = torch.cuda.Event()
            ev.record(main_s)
            for s in streams:
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    chain(n, cycles)
            for s in streams:
                e = torch.cuda.Event()
                e.record(s)
                main_s.wait_event(e)

        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream()
        with torch.cuda.stream(cap):
            g.capture_begin()
            ev = torch.cuda.Event()
            ev.record(cap)
            keep = [ev]
            for s in streams:
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    chain(n, cycles)
            for s in streams:
                e = torch.cuda.Event()
                e.record(s)
                keep.append(e)
                cap.wait_event(e)
            g.capture_end()
        print(f"branches={branches} eager_ms={timed(eager):.3f} "
              f"graph_ms={timed(g.replay):.3f}", flush=True)


if __name__ == "__main__":
    main()
