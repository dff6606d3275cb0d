"""``vixen``: run ONE party of a computation in this process (reference
``moose/src/bin/vixen/main.rs``: per-party runner with a role assignment and host list,
raw-TCP networking).

Two transports:

* ``--transport rccl`` (default): launch one process per identity with any launcher that
  sets the torch.distributed environment (``torchrun``, Slurm, ...); rank r plays role r
  (RCCL between GPUs when CUDA is visible, gloo otherwise)::

      torchrun --nproc-per-node 3 --master-addr 127.0.0.1 -m moose_amd.cli.vixen \\
          --comp examples/dot.moose --roles alice,bob,carole [--compile] [--arg x=x.npy]

* ``--transport tcp``: no process group; the native TCP networking connects the
  identities listed in ``--hosts`` (JSON ``{"alice": "10.0.0.1:4000", ...}``, the
  reference's flag) and the native dataflow scheduler runs this identity's operations of
  a lowered computation -- the cross-node mode::

      vixen --transport tcp --identity alice --hosts '{"alice": ...}' --comp plan.moose

Outputs the identity owns are printed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _load_args(items):
    from moose_amd.utils.storage import load_from_path

    args = {}
    for it in items:
        k, _, p = it.partition("=")
        args[k] = load_from_path(p, None)
    return args


def _print_outputs(ident, outs, elapsed):
    for k in sorted(outs):
        v = outs[k]
        if hasattr(v, "detach"):
            v = v.detach().cpu().numpy()
        print(f"[{ident}] {k} = {np.array2string(np.asarray(v), threshold=20)}")
    print(f"[{ident}] elapsed_us = {elapsed}", flush=True)


def _run_tcp(a, comp, args) -> int:
    from moose_amd.compiler import passes
    from moose_amd.runtime.dataflow import TcpTransport
    from moose_amd.runtime.distributed import _host_numpy
    from moose_amd.runtime.graph_executor import GraphExecutor
    from moose_amd.runtime.local import arg_specs_of

    hosts = json.loads(a.hosts)
    if a.identity not in hosts:
        raise SystemExit(f"identity {a.identity} is not in --hosts")
    if not passes.is_lowered(comp):
        comp = passes.compile(comp, arg_specs=arg_specs_of(args), fixedpoint_ring=a.ring)
    elif not any(op.kind == "Send" for op in comp.operations):
        comp = passes.compile(comp, ["networking", "toposort"])
    device = a.device or "cpu"
    tr = TcpTransport(a.identity, hosts, session_id=a.session_id, certs_dir=a.certs).start()
    try:
        ex = GraphExecutor(device, identity=a.identity, transport=tr, timeout_s=a.timeout)
        t0 = time.perf_counter()
        outs = ex.run(comp, args)
        elapsed = int((time.perf_counter() - t0) * 1e6)
    finally:
        tr.close()
    _print_outputs(a.identity, {k: _host_numpy(v) for k, v in outs.items()}, elapsed)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="vixen", description=__doc__.splitlines()[0])
    ap.add_argument("--comp", required=True)
    ap.add_argument("-i", "--input-format", default="textual", choices=("textual", "msgpack"))
    ap.add_argument("--transport", default="rccl", choices=("rccl", "tcp"))
    ap.add_argument("--roles", help="comma-separated role per rank (rccl transport)")
    ap.add_argument("--identity", "--placement", dest="identity",
                    help="this process's identity (tcp transport)")
    ap.add_argument("--role-assignment", default=None,
                    help='JSON {"role": "identity"} applied to the computation\'s roles')
    ap.add_argument("--hosts", help='JSON {"identity": "host:port"} (tcp transport)')
    ap.add_argument("--session-id", default="vixen")
    ap.add_argument("--certs", help="mutual TLS: directory with <identity>.crt/.key, ca.crt")
    ap.add_argument("--timeout", type=float, default=300.0, help="session deadline (s)")
    ap.add_argument("--device", default=None)
    ap.add_argument("--compile", action="store_true")
    ap.add_argument("--arg", action="append", default=[], help="name=path.npy")
    ap.add_argument("--ring", type=int, default=128, choices=(64, 128))
    a = ap.parse_args(argv)
    from moose_amd.cli.common import read_computation

    comp = read_computation(a.comp, a.input_format)
    if a.role_assignment:
        comp = comp.with_roles(json.loads(a.role_assignment))
    args = _load_args(a.arg)
    if a.transport == "tcp":
        if not (a.identity and a.hosts):
            ap.error("--transport tcp needs --identity and --hosts")
        return _run_tcp(a, comp, args)
    if not a.roles:
        ap.error("--transport rccl needs --roles")

    import torch
    import torch.distributed as dist

    from moose_amd.runtime.distributed import party_device
    from moose_amd.runtime.distributed import run_spmd
    from moose_amd.runtime.local import arg_specs_of

    roles = a.roles.split(",")
    rank = int(os.environ["RANK"])
    backend = "nccl" if torch.cuda.device_count() >= len(roles) else "gloo"
    device = party_device(backend, int(os.environ.get("LOCAL_RANK", rank)))
    if device.type == "cuda":
        torch.cuda.set_device(device)
    dist.init_process_group(backend)
    if a.compile:
        from moose_amd.compiler import passes

        comp = passes.compile(comp, arg_specs=arg_specs_of(args), fixedpoint_ring=a.ring)
    outs, _, elapsed = run_spmd(comp, args, roles, rank=rank, device=device,
                                fixedpoint_ring=a.ring)
    _print_outputs(roles[rank], outs, elapsed)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
