"""Does a communication kernel on a second stream get CUs while the CRT GEMM runs?
(the bench's two-stream overlap assumes it does.)

The stand-in for an RCCL point-to-point channel kernel is ``mx_copy_channels``: a copy of
one share-tensor message (4096^2 Z_2^128 = 256 MiB) with 16 workgroups.  Measured, each
five times after a warm-up, with HIP events (and, under ``rocprofv3 --kernel-trace``, the
kernels' own start/end times -- ``--summarize`` reads them):

* the 4096^2 Z_2^128 rolled-pair CRT product alone (prep, GEMM, reconstruction);
* the copy alone;
* both: the product on stream A, the copy on stream B issued 3 ms later (inside the GEMM);
* the same with stream A restricted to all but k CUs (``hipExtStreamCreateWithCUMask``), k
  = 8, 16, 32, taken either from the top of the mask or evenly from every 32-CU word.

GPU_MAX_HW_QUEUES is 8 here, as bench.py sets it for multi-GPU runs (streams that share a
hardware queue serialise; profiles/r3_stream_concurrency.md).
"""
import argparse
import csv
import glob
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _mask(ncu, free, spread):
    words = [0xFFFFFFFF] * ((ncu + 31) // 32)
    if spread:  # k / words CUs off the top of every word
        per = free // len(words)
        for w in range(len(words)):
            for j in range(per):
                words[w] &= ~(1 << (31 - j))
    else:
        for j in range(free):
            b = ncu - 1 - j
            words[b // 32] &= ~(1 << (b % 32))
    return words


def run(out_path, reps=5, size=4096):
    import ctypes

    import torch

    from moose_amd.ops import native as nat
    from moose_amd.ops import ring as R

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lib = nat.lib()
    g = torch.Generator(device="cpu").manual_seed(1)

    def rand(shape):
        return R.RT(torch.randint(-2**62, 2**62, shape + (2,), generator=g).to(dev), 128)

    x0, y0, y1 = rand((3, size, size)), rand((3, size, size)), rand((3, size, size))
    nbytes = size * size * 16
    src = torch.empty(nbytes // 8, dtype=torch.int64, device=dev).random_()
    dst = torch.empty_like(src)
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count

    def product():
        return R.dot_cross_pair(x0, y0, y1, 1)

    def copy(stream):
        rc = lib.mx_copy_channels(nat.ptr(dst), nat.ptr(src), nbytes, 16,
                                  ctypes.c_void_p(stream.cuda_stream))
        assert rc == 0, rc

    def timed(fn, stream):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            a.record()
            fn()
            b.record()
        return a, b

    sb = torch.cuda.Stream(dev)
    res = {"device": torch.cuda.get_device_name(dev), "cus": ncu, "reps": reps,
           "message_mib": nbytes >> 20, "copy_workgroups": 16, "arms": {}}

    def arm(name, stream_a, concurrent):
        prod, cp = [], []
        for i in range(reps + 1):
            torch.cuda.synchronize()
            ea = timed(product, stream_a) if stream_a is not None else None
            if concurrent or stream_a is None:
                if ea is not None:
                    time.sleep(0.003)  # the copy arrives while the GEMM runs
                eb = timed(lambda: copy(sb), sb)
            torch.cuda.synchronize()
            if i:
                if ea is not None:
                    prod.append(ea[0].elapsed_time(ea[1]))
                if concurrent or stream_a is None:
                    cp.append(eb[0].elapsed_time(eb[1]))
        rec = {}
        if prod:
            rec["product_ms"] = sorted(prod)[len(prod) // 2]
        if cp:
            rec["copy_ms"] = sorted(cp)[len(cp) // 2]
        res["arms"][name] = rec
        print(name, rec, flush=True)

    sa = torch.cuda.Stream(dev)
    arm("product_alone", sa, False)
    arm("copy_alone", None, True)
    arm("both", sa, True)
    masked = []
    for free in (8, 16, 32):
        for spread in (False, True):
            words = _mask(ncu, free, spread)
            arr = (ctypes.c_uint32 * len(words))(*words)
            out = ctypes.c_void_p()
            if lib.mx_stream_cumask(arr, len(words), ctypes.byref(out)) != 0:
                res["arms"][f"mask{free}"] = {"error": "hipExtStreamCreateWithCUMask failed"}
                continue
            ms = torch.cuda.ExternalStream(out.value, device=dev)
            masked.append(out)
            tag = f"cumask_free{free}_{'spread' if spread else 'top'}"
            arm(tag + "_alone", ms, False)
            arm(tag + "_both", ms, True)
    torch.cuda.synchronize()
    for m in masked:
        lib.mx_stream_destroy(m)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


def summarize(trace_dir):
    """Kernel-trace view: for each copy kernel, when it started relative to the CRT GEMM
    that was running (negative: before it ended = co-resident)."""
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    gemms = sorted((s, e) for s, e, n in ks if "k_crt_gemm16" in n)
    copies = sorted((s, e) for s, e, n in ks if "k_copy_channels" in n)
    out = []
    for s, e in copies:
        g = [(gs, ge) for gs, ge in gemms if gs <= s <= ge]
        if g:
            gs, ge = g[0]
            out.append({"copy_start_after_gemm_start_us": (s - gs) / 1e3,
                        "copy_end_before_gemm_end_us": (ge - e) / 1e3,
                        "copy_us": (e - s) / 1e3, "gemm_us": (ge - gs) / 1e3,
                        "overlapped": e < ge})
        else:
            after = [(gs, ge) for gs, ge in gemms if ge <= s]
            out.append({"copy_us": (e - s) / 1e3, "overlapped": False,
                        "started_after_gemm_end_us": (s - after[-1][1]) / 1e3 if after else None})
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/coresid.json")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--summarize", default=None, help="rocprofv3 output directory")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a.out, a.reps)
