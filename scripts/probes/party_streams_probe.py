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
    ser, _ = compose(pt, dag=False)
    ref_bufs, ref_srcs, ref_out = replay(pt, ser, args)
    cps = [a for a in pt.actions if a[0] == "cp"]
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
        same = all(np.array_equal(np.asarray(out[h][k]), np.asarray(ref_out[k]))
                   for h in out for k in out[h] if k in ref_out)
        rec[f"replay{rep}"] = {
            "outputs_equal": same, "messages_differing": ndiff, "first_diff": first,
            "epochs": [int(e.item()) for e in pt._epochs],
            "errs": [int(e.item()) for e in pt._errs],
            "flags": [f.tolist() for f in pt._flags]}
        print(json.dumps({f"replay{rep}": rec[f"replay{rep}"]}), flush=True)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
