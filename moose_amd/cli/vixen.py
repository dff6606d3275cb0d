"""``vixen``: run ONE party of a computation in this process (reference
``moose/src/bin/vixen/main.rs``: per-party runner with a role assignment and host list).

Launch one process per identity with any launcher that sets the torch.distributed
environment (``torchrun``, Slurm, ...)::

    torchrun --nproc-per-node 3 --master-addr 127.0.0.1 -m moose_amd.cli.vixen \\
        --comp examples/dot.moose --roles alice,bob,carole [--compile] [--arg x=x.npy]

Rank r plays role r (RCCL between GPUs when CUDA is visible, gloo otherwise); outputs the
identity owns are printed.  Lowered graphs run on the per-identity graph executor,
logical ones on the SPMD session.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="vixen", description=__doc__.splitlines()[0])
    ap.add_argument("--comp", required=True)
    ap.add_argument("-i", "--input-format", default="textual", choices=("textual", "msgpack"))
    ap.add_argument("--roles", required=True, help="comma-separated role per rank")
    ap.add_argument("--compile", action="store_true")
    ap.add_argument("--arg", action="append", default=[], help="name=path.npy")
    ap.add_argument("--ring", type=int, default=128, choices=(64, 128))
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    from moose_amd.cli.common import read_computation
    from moose_amd.runtime.distributed import party_device
    from moose_amd.runtime.distributed import run_spmd
    from moose_amd.runtime.local import arg_specs_of
    from moose_amd.utils.storage import load_from_path

    roles = a.roles.split(",")
    rank = int(os.environ["RANK"])
    backend = "nccl" if torch.cuda.device_count() >= len(roles) else "gloo"
    device = party_device(backend, int(os.environ.get("LOCAL_RANK", rank)))
    if device.type == "cuda":
        torch.cuda.set_device(device)
    dist.init_process_group(backend)
    comp = read_computation(a.comp, a.input_format)
    args = {}
    for it in a.arg:
        k, _, p = it.partition("=")
        args[k] = load_from_path(p, None)
    if a.compile:
        from moose_amd.compiler import passes

        comp = passes.compile(comp, arg_specs=arg_specs_of(args), fixedpoint_ring=a.ring)
    outs, _, elapsed = run_spmd(comp, args, roles, rank=rank, device=device,
                                fixedpoint_ring=a.ring)
    for k in sorted(outs):
        print(f"[{roles[rank]}] {k} = {np.array2string(np.asarray(outs[k]), threshold=20)}")
    print(f"[{roles[rank]}] elapsed_us = {elapsed}")
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
