"""Where do the in-process parties' message buffers live?  (The composed-as-DAG hazard: a
copy that runs beside a THIRD party's segment corrupts it, so some memory is shared between
parties.)  Seeded LR parties on one GPU, tapes captured as for the composed replay; every
CommStep payload / landing buffer is located in torch's memory snapshot (which private
graph pool, or the default pool) and checked for overlaps with the buffers of the other
parties and with the other messages of its own party."""
import json
import os
import sys

sys.path.insert(0, os.getcwd())


def main():
    import torch

    from moose_amd.models.predictors.tutorial import logistic_regression_tutorial
    from moose_amd.parallel.transport import CommStep
    from moose_amd.runtime.local import LocalMooseRuntime

    ids = ["alice", "bob", "carole"]
    tm = logistic_regression_tutorial(128)
    args = {"x": tm.x_test}
    rt = LocalMooseRuntime(ids, device_map={i: "cuda:0" for i in ids}, seed=11, use_graphs=True,
                           timeout=60)
    for _ in range(2):
        rt.evaluate_computation(tm.computation, args)
    (_, pt), = rt._party_tapes.values()
    items = []  # (lo, hi, party, kind, step, j)
    for p, tape in enumerate(pt.tapes):
        k = 0
        for st in tape.steps:
            if not isinstance(st, CommStep):
                continue
            for j, (t, _dst) in enumerate(st.sends):
                items.append((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size(), p,
                              "send", k, j))
            for j, (b, _src) in enumerate(st.recvs):
                items.append((b.data_ptr(), b.data_ptr() + b.numel() * b.element_size(), p,
                              "recv", k, j))
            k += 1
    snap = torch.cuda.memory_snapshot()
    segs = [(s["address"], s["address"] + s["total_size"], str(s.get("segment_pool_id")))
            for s in snap]

    def pool_of(a):
        for lo, hi, pid in segs:
            if lo <= a < hi:
                return pid
        return "outside-torch"

    pools = {}
    for lo, hi, p, kind, k, j in items:
        pools.setdefault(p, {}).setdefault(pool_of(lo), 0)
        pools[p][pool_of(lo)] += 1
    items.sort()
    cross, same = [], []
    for i in range(len(items)):
        for m in range(i + 1, len(items)):
            a, b = items[i], items[m]
            if b[0] >= a[1]:
                break
            rec = {"a": a[2:], "b": b[2:], "a_range": [a[0], a[1]], "b_range": [b[0], b[1]]}
            (cross if a[2] != b[2] else same).append(rec)
    out = {"messages": len(items), "pools_per_party": {str(p): v for p, v in pools.items()},
           "cross_party_overlaps": len(cross), "same_party_overlaps": len(same),
           "cross_examples": cross[:8], "same_examples": same[:8]}
    print(json.dumps(out, default=str), flush=True)


if __name__ == "__main__":
    main()
