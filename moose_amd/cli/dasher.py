"""``dasher``: simulate every role of a computation in one process.

Parity: reference ``moose/src/bin/dasher/main.rs:1-117`` (runs a compiled computation
on an in-process multi-role session and prints outputs).  Logical computations run on
the stacked single-device session; lowered ones on the graph executor::

    dasher COMPUTATION [-i textual|msgpack] [--compile] [--arg name=file.npy ...]
           [--device cuda|cpu] [--ring 64|128]
    dasher --session FILE.session [--arg name=file.npy ...] [--backend nccl|gloo]

``--session`` runs a filesystem-choreography session file with one worker process per
(replica, role) on this node, honouring its ``gpu``/``gpus`` pinning and ``replicas``.
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

from moose_amd.cli.common import FORMATS
from moose_amd.cli.common import read_computation


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="dasher", description=__doc__.splitlines()[0])
    ap.add_argument("input", nargs="?")
    ap.add_argument("--session", default=None, help="run a .session file (multi-process)")
    ap.add_argument("--backend", default=None)
    ap.add_argument("-i", "--input-format", default="textual", choices=FORMATS)
    ap.add_argument("--compile", action="store_true", help="lower before running")
    ap.add_argument("--arg", action="append", default=[], help="name=path.npy")
    ap.add_argument("--device", default=None)
    ap.add_argument("--ring", type=int, default=128, choices=(64, 128))
    a = ap.parse_args(argv)
    from moose_amd.runtime.local import LocalMooseRuntime
    from moose_amd.utils.storage import load_from_path

    if a.session:
        from moose_amd.runtime.choreography import run_session_file

        extra = {}
        for it in a.arg:
            k, _, p = it.partition("=")
            extra[k] = load_from_path(p, None)
        outs, timings = run_session_file(a.session, extra, backend=a.backend)
        for k in sorted(outs):
            print(f"{k} = {np.array2string(np.asarray(outs[k]), threshold=20)}")
        print(f"elapsed_us = {timings}")
        return 0
    if not a.input:
        ap.error("a computation (or --session) is required")
    comp = read_computation(a.input, a.input_format)
    args = {}
    for it in a.arg:
        k, _, p = it.partition("=")
        args[k] = load_from_path(p, None)
    roles = sorted({r for op in comp.operations for r in
                    ((op.placement.owner,) if hasattr(op.placement, "owner") else op.placement.owners)})
    rt = LocalMooseRuntime(roles, device=a.device, fixedpoint_ring=a.ring)
    if a.compile:
        from moose_amd.compiler import passes

        outs = rt.evaluate_computation(comp, args, compiler_passes=passes.DEFAULT_PASSES)
    else:
        outs = rt.evaluate_compiled(comp, args)
    for k in sorted(outs):
        print(f"{k} = {np.array2string(np.asarray(outs[k]), threshold=20)}")
    print(f"elapsed_us = {rt.last_timings}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
