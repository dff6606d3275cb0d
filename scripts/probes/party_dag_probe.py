"""Why did the composed party graph as a DAG (round 4's MOOSEX_PARTY_GRAPH_DAG=1) not
reproduce the eager values?  

Seeded in-process parties on ONE GPU (LR tutorial model): the per-party tapes are composed
(a) in the serial issue order and (b) as the round-4 DAG (program order per party, send ->
receive copy edges, copy -> sender's-next-segment edges).  Both replays use the same seeded
keys, so every message (landing buffer) must be bitwise equal.  The probe prints, in
schedule order, the first message that differs and the state of its sender's payload
tensor, and repeats the DAG with variants that each remove one suspect."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.getcwd())


def compose(pt, dag, extra_edges=None):
    from moose_amd.ops import native as nat

    n = len(pt.tapes)
    kinds, child, dst, src, nbytes, deps = [], [], [], [], [], []
    last = [None] * n
    sent_at = {}
    reading = [[] for _ in range(n)]
    cp_nodes = []
    for a in pt.actions:
        p = a[1]
        if a[0] == "g":
            kinds.append(0)
            child.append(a[2].raw_cuda_graph())
            dst.append(0)
            src.append(0)
            nbytes.append(0)
            deps.append(sorted(set(([last[p]] if last[p] is not None else []) + reading[p])))
            reading[p] = []
            last[p] = len(kinds) - 1
        elif a[0] == "rec":
            sent_at[id(a[2])] = (last[p], p)
        else:
            _, p, s, t, buf, ev = a
            at, sender = sent_at.get(id(ev), (None, None))
            d = [x for x in (last[p], at) if x is not None]
            kinds.append(1)
            child.append(0)
            dst.append(buf.data_ptr())
            src.append(t.data_ptr())
            nbytes.append(t.numel() * t.element_size())
            deps.append(sorted(set(d)))
            last[p] = len(kinds) - 1
            cp_nodes.append(len(kinds) - 1)
            if sender is not None and sender != p:
                reading[sender].append(last[p])
    m = len(kinds)
    if not dag:
        deps = [sorted(set(d) | ({i - 1} if i else set())) for i, d in enumerate(deps)]
    if extra_edges is not None:
        deps = extra_edges(deps, kinds)
    off = [0]
    flat = []
    for d in deps:
        flat += d
        off.append(len(flat))
    arr = lambda ty, xs: (ty * max(1, len(xs)))(*xs)  # noqa: E731
    g, ex = ctypes.c_void_p(), ctypes.c_void_p()
    rc = nat.lib().mx_graph_compose(
        m, arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child), arr(ctypes.c_void_p, dst),
        arr(ctypes.c_void_p, src), arr(ctypes.c_int64, nbytes), arr(ctypes.c_int, off),
        arr(ctypes.c_int, flat), ctypes.byref(g), ctypes.byref(ex))
    assert rc == 0, rc
    return ex, m


def replay(pt, ex, args):
    import torch

    from moose_amd.ops import native as nat

    s = pt.streams[0]
    with torch.cuda.stream(s):
        for tape in pt.tapes:
            tape.copy_arguments(args)
            tape._fill_keys()
        nat.check(nat.lib().mx_graph_launch(ex, s.cuda_stream), "launch")
    torch.cuda.synchronize()
    bufs = [a[4].clone() for a in pt.actions if a[0] == "cp"]
    srcs = [a[3].clone() for a in pt.actions if a[0] == "cp"]
    outs = {}
    with torch.cuda.stream(s):
        for p, tape in enumerate(pt.tapes):
            outs.update(tape._decode(tape.interp, tape.sess, tape.outs))
    return bufs, srcs, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    ids = ["alice", "bob", "carole"]
    tm = logistic_regression_tutorial(128)
    args = {"x": tm.x_test}
    rt = LocalMooseRuntime(ids, device_map={i: "cuda:0" for i in ids}, seed=11, use_graphs=True,
                           timeout=60)
    want = None
    for _ in range(3):
        want = rt.evaluate_computation(tm.computation, args)
    (_, pt), = rt._party_tapes.values()
    cps = [x for x in pt.actions if x[0] == "cp"]
    from moose_amd.ops import native as nat

    # GEMM workspace lookups that fell back to a slot shared between streams (round 4 had
    # 8 slots per device: parties' segments replayed concurrently could share scratch)
    rec = {"actions": len(pt.actions), "copies": len(cps),
           "workspace_shared_lookups": int(nat.lib().mx_workspace_shared_count())}
    ser, _ = compose(pt, dag=False)
    ref_bufs, ref_srcs, ref_out = replay(pt, ser, args)
    rec["serial_vs_eager"] = all(np.array_equal(np.asarray(ref_out[k]), np.asarray(want[k]))
                                 for k in want)

    def first_diff(bufs, srcs):
        for i, (b, rb) in enumerate(zip(bufs, ref_bufs)):
            if not torch.equal(b, rb):
                act = cps[i]
                return {"copy_index": i, "receiver": act[1], "sender": act[2],
                        "bytes": act[3].numel() * act[3].element_size(),
                        "sender_payload_final_equals_ref": bool(torch.equal(srcs[i],
                                                                            ref_srcs[i])),
                        "landing_equals_ref_payload": bool(torch.equal(b, ref_srcs[i]))}
        return None

    variants = {"dag": None}

    def chain_copies(deps, kinds):  # every copy after the previous node in issue order
        return [sorted(set(d) | ({i - 1} if i and kinds[i] == 1 else set()))
                for i, d in enumerate(deps)]

    def chain_segments(deps, kinds):  # every segment after the previous node
        return [sorted(set(d) | ({i - 1} if i and kinds[i] == 0 else set()))
                for i, d in enumerate(deps)]

    variants["dag+copies_in_order"] = chain_copies
    variants["dag+segments_in_order"] = chain_segments
    for name, extra in variants.items():
        ex, m = compose(pt, dag=True, extra_edges=extra)
        res = []
        for _ in range(a.reps):
            bufs, srcs, out = replay(pt, ex, args)
            same = all(np.array_equal(np.asarray(out[k]), np.asarray(ref_out[k]))
                       for k in ref_out)
            res.append({"outputs_equal": same, "first_diff": first_diff(bufs, srcs)})
        rec[name] = res
        print(json.dumps({name: res}), flush=True)
    # device time of one launch (launch -> synchronize), median of 20: serial vs DAG
    import time

    def timed(ex):
        s = pt.streams[0]
        ts = []
        for _ in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nat.check(nat.lib().mx_graph_launch(ex, s.cuda_stream), "launch")
            s.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        return sorted(ts)[10]

    ex_dag, m_dag = compose(pt, dag=True)
    rec["launch_ms_serial"] = timed(ser)
    rec["launch_ms_dag"] = timed(ex_dag)
    rec["nodes"] = m_dag
    print(json.dumps({k: rec[k] for k in ("launch_ms_serial", "launch_ms_dag", "nodes")}),
          flush=True)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
