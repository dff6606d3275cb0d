"""In-MPC AES-128 decryption latency (the Decrypt op on a replicated placement, as in the
reference's AesWrapper predictors): a secret-shared key decrypts n ciphertexts of
fixed(24,40) values; one JSON line with p50 latency, AND-gate count and AND depth of the
circuit.  MOOSEX_AES_SBOX=algebraic selects the round-1 S-box circuit (x^254 by four
GF(2^8) products) for before/after numbers."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16, help="ciphertexts (fixed-point values)")
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--device", default=None)
    a = ap.parse_args()
    import torch

    from moose_amd.ir.computation import ReplicatedPlacement
    from moose_amd.ops import ring as R
    from moose_amd.protocols import aes
    from moose_amd.protocols import replicated as rep
    from moose_amd.runtime.session import HV
    from moose_amd.runtime.session import StackedSession

    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    key = os.urandom(16)
    vals = np.linspace(-100, 100, a.n)
    ct = aes.encrypt_fixed(key, vals, 40)
    kbits = np.unpackbits(np.frombuffer(key, dtype=np.uint8))
    plc = ReplicatedPlacement(("a", "b", "c"))
    lc = aes.levelled_aes()

    def once():
        sess = StackedSession(dev)
        K = rep.share(sess, plc, HV("a", R.RT(torch.as_tensor(kbits).to(dev), 1)), kind="bool")
        C = rep.share(sess, plc, HV("b", R.RT(torch.as_tensor(ct).to(dev), 1)), kind="bool")
        T = aes.rep_decrypt(sess, plc, K, C)
        out = rep.reveal(sess, T, "c")
        if dev != "cpu":
            torch.cuda.synchronize()
        return out

    for _ in range(a.warmup):
        out = once()
    lat = []
    for _ in range(a.runs):
        t0 = time.perf_counter()
        out = once()
        lat.append(time.perf_counter() - t0)
    err = float(np.abs(R.decode(out.v, 40).cpu().numpy() - vals).max())
    lat = np.sort(np.asarray(lat)) * 1e3
    print(json.dumps({
        "metric": "in-MPC AES-128 decrypt p50 latency", "value": float(np.median(lat)),
        "unit": "ms", "n_ciphertexts": a.n, "runs": a.runs, "device": dev,
        "and_gates": lc.and_count, "and_depth": lc.depth,
        "sbox": os.environ.get("MOOSEX_AES_SBOX", "boyar-peralta"), "max_abs_err": err,
    }), flush=True)


if __name__ == "__main__":
    main()
