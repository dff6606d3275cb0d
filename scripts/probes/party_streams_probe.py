"""Per-party graphs on three streams (MOOSEX_PARTY_STREAMS=1, threads.py _build_streams):
which message first differs from the serial composed replay of the SAME tapes (seeded keys:
every landing buffer must be bitwise equal), and the state of the device-side flags,
epochs and error words after the replay."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "scripts", "probes"))


def main():
    os.environ["MOOSEX_PARTY_STREAMS"] = "1"
    os.environ["MOOSEX_PARTY_STREAMS_SHADOW"] = "1"
    os.environ["MOOSEX_DEBUG_KEEP"] = "1"
    import numpy as np
    import torch

    from party_dag_probe import compose
    from party_dag_probe import replay
    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.runtime.local import LocalMooseRuntime

    ids = ["alice", "bob", "carole"]
    tm = logistic_regression_tutorial(128)
    args = {"x": tm.x_test}
    rt = LocalMooseRuntime(ids, device_map={i: "cuda:0" for i in ids}, seed=11, use_graphs=True,
                           timeout=60)
    for _ in range(2):  # warm-up (eager), capture + first replay
        rt.evaluate_computation(tm.computation, args)
    (_, pt), = rt._party_tapes.values()
    rec = {"streams_mode": pt._party_graphs is not None}
    from moose_amd.ops import native as nat0

    outdir = os.environ.get("PROBE_OUT")
    if outdir:  # the party graphs as DOT (kernel arguments) + torch's memory segments
        for q, (g, _ex) in enumerate(pt._party_graphs):
            nat0.lib().mx_graph_dot(g, os.path.join(outdir, f"party{q}.dot").encode(), 1)
        segs = [{"address": x["address"], "size": x["total_size"],
                 "pool": str(x.get("segment_pool_id")),
                 "blocks": [(b["size"], b["state"]) for b in x["blocks"]]}
                for x in torch.cuda.memory_snapshot()]
        with open(os.path.join(outdir, "segments.json"), "w") as fh:
            json.dump({"segments": segs,
                       "keys": [t.keys.t.data_ptr() for t in pt.tapes],
                       "streams": [str(t.stream) for t in pt.tapes]}, fh)
    ser, _ = compose(pt, dag=False)
    ref_bufs, ref_srcs, ref_out = replay(pt, ser, args)
    cps = [a for a in pt.actions if a[0] == "cp"]
    pair_k, cnt = [], {}
    for a in cps:  # (sender, receiver, k-th message of that pair)
        kk = cnt.get((a[2], a[1]), 0)
        cnt[(a[2], a[1])] = kk + 1
        pair_k.append((a[2], a[1], kk, a[3].numel() * a[3].element_size()))
    rec["copies_pair_k"] = pair_k
    for rep in range(3):
        out = pt.replay(args)
        torch.cuda.synchronize()
        bufs = [a[4].clone() for a in cps]
        first = None
        ndiff = 0
        for i, (b, rb) in enumerate(zip(bufs, ref_bufs)):
            if not torch.equal(b, rb):
                ndiff += 1
                if first is None:
                    a = cps[i]
                    first = {"copy_index": i, "receiver": a[1], "sender": a[2],
                             "bytes": a[3].numel() * a[3].element_size(),
                             "landing_equals_payload_now": bool(torch.equal(b, a[3])),
                             "payload_equals_ref_payload": bool(torch.equal(a[3], ref_srcs[i]))}
        # landing buffers as seen right after their waits vs the serial reference
        ref_of = {a[4].data_ptr(): rb for a, rb in zip(cps, ref_bufs)}
        sh_bad = [i for i, (buf, sh) in enumerate(pt._shadows)
                  if not torch.equal(sh, ref_of[buf.data_ptr()])]
        premature = [cps_i for cps_i, (buf, sh) in
                     ((next(i for i, a in enumerate(cps) if a[4].data_ptr() == b.data_ptr()),
                       (b, sh)) for b, sh in pt._shadows) if not torch.equal(sh, buf)]
        sh_first = None
        if sh_bad:
            buf, sh = pt._shadows[sh_bad[0]]
            sh_first = {"shadow_index": sh_bad[0], "final_equals_ref":
                        bool(torch.equal(buf, ref_of[buf.data_ptr()])),
                        "copy_index": next(i for i, a in enumerate(cps)
                                           if a[4].data_ptr() == buf.data_ptr())}
        same = all(np.array_equal(np.asarray(out[h][k]), np.asarray(ref_out[k]))
                   for h in out for k in out[h] if k in ref_out)
        rec[f"replay{rep}"] = {
            "outputs_equal": same, "messages_differing": ndiff, "first_diff": first,
            "shadows": len(pt._shadows), "shadows_differing": len(sh_bad),
            "shadow_not_final": sorted(premature)[:10],
            "earliest_bad_copy": min((next(i for i, a in enumerate(cps)
                                           if a[4].data_ptr() == pt._shadows[j][0].data_ptr())
                                      for j in sh_bad), default=None),
            "first_shadow_diff": sh_first,
            "epochs": [int(e.item()) for e in pt._epochs],
            "errs": [int(e.item()) for e in pt._errs],
            "flags": [f.tolist() for f in pt._flags]}
        print(json.dumps({f"replay{rep}": rec[f"replay{rep}"]}), flush=True)
    # the per-party graphs' push tables against the serial schedule's copies
    rows = set()
    for tab in pt._tables:
        if tab.dtype != torch.int64 or tab.numel() % 5:
            continue
        v = tab.view(-1, 5).tolist()
        rows |= {(a % (1 << 64), b % (1 << 64), c) for a, b, c, _f, _p in v}
    want = {(a[3].data_ptr(), a[4].data_ptr(), a[3].numel() * a[3].element_size()) for a in cps}
    rec["push_rows"] = len(rows)
    rec["copies"] = len(want)
    rec["rows_not_in_schedule"] = len(rows - want)
    rec["schedule_not_in_rows"] = len(want - rows)
    print(json.dumps({k: rec[k] for k in ("push_rows", "copies", "rows_not_in_schedule",
                                          "schedule_not_in_rows")}), flush=True)
    # the same node kinds as the per-party graphs (segments + k_push with a flag per
    # message), but ONE chain in the serial schedule's order on one stream: separates the
    # push / flag mechanism and the message mapping from the concurrency of three graphs
    import ctypes

    from moose_amd.ops import native as nat

    dev = pt.devices[0]
    scratch_flag = torch.zeros(len(cps) + 1, dtype=torch.int32, device=dev)
    scratch_pieces = torch.zeros(len(cps) + 1, dtype=torch.int32, device=dev)
    epoch = torch.zeros(1, dtype=torch.int64, device=dev)
    kinds, child, p0, p1, p2, i0, i64, keep = [5], [0], [epoch.data_ptr()], [0], [0], [0], [0], []
    ci = 0
    for a in pt.actions:
        if a[0] == "g":
            kinds.append(0); child.append(a[2].raw_cuda_graph()); p0.append(0); p1.append(0)
            p2.append(0); i0.append(0); i64.append(0)
        elif a[0] == "cp":
            t, buf = a[3], a[4]
            nb = t.numel() * t.element_size()
            row = [t.data_ptr(), buf.data_ptr(), nb, scratch_flag.data_ptr() + 4 * ci,
                   scratch_pieces.data_ptr() + 4 * ci]
            tab = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in row],
                               dtype=torch.int64, device=dev)
            keep.append(tab)
            kinds.append(6); child.append(0); p0.append(tab.data_ptr()); p1.append(epoch.data_ptr())
            p2.append(0); i0.append(1); i64.append(nb)
            ci += 1
    k = len(kinds)
    arr = lambda ty, xs: (ty * k)(*xs)  # noqa: E731
    g, ex = ctypes.c_void_p(), ctypes.c_void_p()
    rc = nat.lib().mx_graph_build_chain(k, arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child),
                                        arr(ctypes.c_void_p, p0), arr(ctypes.c_void_p, p1),
                                        arr(ctypes.c_void_p, p2), arr(ctypes.c_int, i0),
                                        arr(ctypes.c_int64, i64), ctypes.byref(g), ctypes.byref(ex))
    rec["serial_push_chain_rc"] = rc
    if rc == 0:
        s0 = pt.streams[0]
        with torch.cuda.stream(s0):
            for tape in pt.tapes:
                tape.copy_arguments(args)
                tape._fill_keys()
            nat.check(nat.lib().mx_graph_launch(ex, s0.cuda_stream), "launch")
        torch.cuda.synchronize()
        bufs = [a[4].clone() for a in cps]
        nd = sum(not torch.equal(b, rb) for b, rb in zip(bufs, ref_bufs))
        first = next((i for i, (b, rb) in enumerate(zip(bufs, ref_bufs))
                      if not torch.equal(b, rb)), None)
        rec["serial_push_chain"] = {"messages_differing": nd, "first_diff": first}
        print(json.dumps({"serial_push_chain": rec["serial_push_chain"]}), flush=True)
    # serial chains in OTHER valid orders (list scheduling with a party priority): an
    # order-dependent result without any concurrency points at an implicit dependency
    from moose_amd.parallel.transport import CommStep

    def order(prio):
        steps = [t.steps for t in pt.tapes]
        ptr = [0] * len(steps)
        sent, got = {}, {}
        seq = []  # ("g", graph) / ("push", rows)
        land = {}
        for q, tape in enumerate(pt.tapes):
            cnt = {}
            for st in tape.steps:
                if isinstance(st, CommStep):
                    for buf, src in st.recvs:
                        k = cnt.get(src, 0)
                        cnt[src] = k + 1
                        land[(src, q, k)] = buf
        done_send = [False] * len(steps)
        while any(ptr[p] < len(steps[p]) for p in range(len(steps))):
            for p in prio:
                if ptr[p] >= len(steps[p]):
                    continue
                st = steps[p][ptr[p]]
                if not isinstance(st, CommStep):
                    seq.append(("g", st))
                    ptr[p] += 1
                    break
                if not done_send[p]:  # a round's sends never wait
                    rows = []
                    for t, dst in st.sends:
                        k = sent.get((p, dst), 0)
                        sent[(p, dst)] = k + 1
                        rows.append((t, land[(p, dst, k)]))
                    if rows:
                        seq.append(("push", rows))
                    done_send[p] = True
                    break
                need = {}
                for _b, src in st.recvs:
                    need[src] = need.get(src, 0) + 1
                if any(sent.get((src, p), 0) < got.get((src, p), 0) + c for src, c in need.items()):
                    continue
                for _b, src in st.recvs:
                    got[(src, p)] = got.get((src, p), 0) + 1
                ptr[p] += 1
                done_send[p] = False
                break
            else:
                # every party blocked on a receive whose send comes later in ITS program:
                # let the first party with pending sends push them (sends never block)
                raise RuntimeError("no runnable step")
        return seq

    def run_order(prio):
        kinds, child, p0, p1, p2, i0, i64 = [5], [0], [epoch.data_ptr()], [0], [0], [0], [0]
        fi = 0
        for kind, v in order(prio):
            if kind == "g":
                kinds.append(0); child.append(v.raw_cuda_graph()); p0.append(0); p1.append(0)
                p2.append(0); i0.append(0); i64.append(0)
                continue
            for t, buf in v:
                nb = t.numel() * t.element_size()
                row = [t.data_ptr(), buf.data_ptr(), nb, scratch_flag.data_ptr() + 4 * (fi % 64),
                       scratch_pieces.data_ptr() + 4 * (fi % 64)]
                fi += 1
                tab = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in row],
                                   dtype=torch.int64, device=dev)
                keep.append(tab)
                kinds.append(6); child.append(0); p0.append(tab.data_ptr())
                p1.append(epoch.data_ptr()); p2.append(0); i0.append(1); i64.append(nb)
        k = len(kinds)
        arr = lambda ty, xs: (ty * k)(*xs)  # noqa: E731
        g, ex = ctypes.c_void_p(), ctypes.c_void_p()
        rc = nat.lib().mx_graph_build_chain(
            k, arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child), arr(ctypes.c_void_p, p0),
            arr(ctypes.c_void_p, p1), arr(ctypes.c_void_p, p2), arr(ctypes.c_int, i0),
            arr(ctypes.c_int64, i64), ctypes.byref(g), ctypes.byref(ex))
        if rc:
            return {"rc": rc}
        s0 = pt.streams[0]
        with torch.cuda.stream(s0):
            for tape in pt.tapes:
                tape.copy_arguments(args)
                tape._fill_keys()
        torch.cuda.synchronize()
        # the per-tape buffers outside the graph pools: nothing in a replay writes them
        watch = {}
        for q, tape in enumerate(pt.tapes):
            watch[f"keys{q}"] = tape.keys.t
            for k, v in tape.static.items():
                if isinstance(v, torch.Tensor) and v.is_cuda:
                    watch[f"static{q}_{k}"] = v
            for j, v in enumerate(tape._stager.dev):
                if v.is_cuda:
                    watch[f"stager{q}_{j}"] = v
        before = {k: v.clone() for k, v in watch.items()}
        with torch.cuda.stream(s0):
            nat.check(nat.lib().mx_graph_launch(ex, s0.cuda_stream), "launch")
        torch.cuda.synchronize()
        changed = [k for k, v in watch.items() if not torch.equal(v, before[k])]
        bufs = [a[4].clone() for a in cps]
        bad = [i for i, (b, rb) in enumerate(zip(bufs, ref_bufs)) if not torch.equal(b, rb)]
        return {"messages_differing": len(bad), "first": bad[0] if bad else None,
                "first_pair_k": pair_k[bad[0]] if bad else None, "changed": changed}

    for prio in ([0, 1, 2], [1, 0, 2], [2, 1, 0], [1, 2, 0], [2, 0, 1]):
        try:
            r = run_order(prio)
        except RuntimeError as e:
            r = {"error": str(e)}
        rec[f"serial_order_{prio}"] = r
        print(json.dumps({f"serial_order_{prio}": r}), flush=True)

    # the same orders with plain memcpy nodes (mx_graph_compose) instead of k_push
    class _Ev:
        pass

    def order_actions(prio):
        acts = []
        land_rev = {}
        for kind, v in order(prio):
            if kind == "g":
                owner = next(q for q, t in enumerate(pt.tapes) if any(v is x for x in t.steps))
                acts.append(("g", owner, v))
            else:
                for t, buf in v:
                    ev = _Ev()
                    owner = next(q for q, tp in enumerate(pt.tapes)
                                 if any(t is x for st in tp.steps if isinstance(st, CommStep)
                                        for x, _ in st.sends))
                    acts.append(("rec", owner, ev))
                    recv = next(q for q, tp in enumerate(pt.tapes)
                                if any(buf is x for st in tp.steps if isinstance(st, CommStep)
                                       for x, _ in st.recvs))
                    acts.append(("cp", recv, owner, t, buf, ev))
        return acts

    for prio in ([1, 0, 2], [2, 1, 0]):
        class _PT:
            pass
        fake = _PT()
        fake.actions = order_actions(prio)
        fake.tapes, fake.streams = pt.tapes, pt.streams
        ex2, _ = compose(fake, dag=False)
        b2, _s2, _o2 = replay(fake, ex2, args)
        bad = [i for i, (b, rb) in enumerate(zip(b2, ref_bufs)) if not torch.equal(b, rb)]
        # b2 is in this order's copy order: map back by landing buffer
        pos = {a[4].data_ptr(): i for i, a in enumerate(cps)}
        got = {a[4].data_ptr(): b for a, b in zip([x for x in fake.actions if x[0] == "cp"], b2)}
        bad = sorted(pos[k] for k, b in got.items() if not torch.equal(b, ref_bufs[pos[k]]))
        r = {"messages_differing": len(bad), "first": bad[0] if bad else None,
             "first_pair_k": pair_k[bad[0]] if bad else None}
        rec[f"memcpy_order_{prio}"] = r
        print(json.dumps({f"memcpy_order_{prio}": r}), flush=True)
    # truncated serial orders: run up to (and including) the push of message ``stop``, then
    # compare the operands the protocol steps recorded at capture (spmd.DEBUG_KEEP)
    from moose_amd.parallel import spmd as SP

    def flat_keep():
        out = []
        for ent in SP.DEBUG_KEEP:
            tensors = []

            def walk(v):
                if isinstance(v, torch.Tensor):
                    tensors.append(v)
                elif isinstance(v, (list, tuple)):
                    for x in v:
                        walk(x)
            walk(ent[2:])
            out.append((ent[0], ent[1], tensors))
        return out

    def run_trunc(prio, stop):
        seq = order(prio)
        target = cps[stop][4].data_ptr()
        cut = next(i for i, (kind, v) in enumerate(seq)
                   if kind == "push" and any(buf.data_ptr() == target for _t, buf in v))
        seq = seq[:cut + 1]
        kinds, child, p0, p1, p2, i0, i64 = [5], [0], [epoch.data_ptr()], [0], [0], [0], [0]
        fi = 0
        for kind, v in seq:
            if kind == "g":
                kinds.append(0); child.append(v.raw_cuda_graph()); p0.append(0); p1.append(0)
                p2.append(0); i0.append(0); i64.append(0)
                continue
            for t, buf in v:
                nb = t.numel() * t.element_size()
                row = [t.data_ptr(), buf.data_ptr(), nb, scratch_flag.data_ptr() + 4 * (fi % 64),
                       scratch_pieces.data_ptr() + 4 * (fi % 64)]
                fi += 1
                tab = torch.tensor([x - (1 << 64) if x >= (1 << 63) else x for x in row],
                                   dtype=torch.int64, device=dev)
                keep.append(tab)
                kinds.append(6); child.append(0); p0.append(tab.data_ptr())
                p1.append(epoch.data_ptr()); p2.append(0); i0.append(1); i64.append(nb)
        k = len(kinds)
        arr = lambda ty, xs: (ty * k)(*xs)  # noqa: E731
        g, ex = ctypes.c_void_p(), ctypes.c_void_p()
        assert nat.lib().mx_graph_build_chain(
            k, arr(ctypes.c_int, kinds), arr(ctypes.c_void_p, child), arr(ctypes.c_void_p, p0),
            arr(ctypes.c_void_p, p1), arr(ctypes.c_void_p, p2), arr(ctypes.c_int, i0),
            arr(ctypes.c_int64, i64), ctypes.byref(g), ctypes.byref(ex)) == 0
        # poison every recorded operand first: what the truncated run does not write shows
        for _n, _who, ts in flat_keep():
            for t in ts:
                t.fill_(-7) if t.dtype.is_floating_point is False else t.fill_(-7.0)
        s0 = pt.streams[0]
        with torch.cuda.stream(s0):
            for tape in pt.tapes:
                tape.copy_arguments(args)
                tape._fill_keys()
            nat.check(nat.lib().mx_graph_launch(ex, s0.cuda_stream), "launch")
        torch.cuda.synchronize()
        return [[t.clone() for t in ts] for _n, _who, ts in flat_keep()]

    if SP.DEBUG_KEEP:
        stop = rec["serial_order_[2, 1, 0]"].get("first")
        if stop is not None:
            A = run_trunc([1, 0, 2], stop)
            B = run_trunc([2, 1, 0], stop)
            meta = flat_keep()
            diffs = []
            for (name, who, ts), ta, tb in zip(meta, A, B):
                d = [j for j, (x, y) in enumerate(zip(ta, tb)) if not torch.equal(x, y)]
                if d:
                    diffs.append({"step": name, "party": who, "operands_differing": d,
                                  "n_operands": len(ts)})
            # where do the kept tensors live relative to the landing buffers / payloads?
            lands = {a[4].data_ptr(): i for i, a in enumerate(cps)}
            pays = {a[3].data_ptr(): i for i, a in enumerate(cps)}
            where = []
            for name, who, ts in meta:
                where.append([name, who, [(lands.get(t.data_ptr()), pays.get(t.data_ptr()))
                                          for t in ts]])
            rec["kept_where"] = where
            print(json.dumps({"kept_where": where}), flush=True)
            rec["trunc_stop"] = stop
            rec["trunc_diffs"] = diffs
            print(json.dumps({"trunc_stop": stop, "trunc_diffs": diffs,
                              "kept": [(n, w, len(t)) for n, w, t in meta]}), flush=True)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
