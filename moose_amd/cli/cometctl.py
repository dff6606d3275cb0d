"""``cometctl``: launch / abort / collect choreographed sessions.

Parity: reference ``moose/src/bin/comet/cometctl.rs:14-145``
(``launch|abort|results|run <session.toml> [--session-id]``)::

    cometctl --store 127.0.0.1:29600 --world 3 run examples/dot.session
    cometctl --store 127.0.0.1:29600 --world 3 shutdown
"""
from __future__ import annotations

import argparse
import os
import sys
import uuid

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cometctl", description=__doc__.splitlines()[0])
    ap.add_argument("--store", default=os.environ.get("MOOSEX_STORE", "127.0.0.1:29600"))
    ap.add_argument("--world", type=int, default=3)
    ap.add_argument("--timeout", type=float, default=3600)
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("launch", "run", "results", "abort"):
        p = sub.add_parser(name)
        p.add_argument("session")
        p.add_argument("--session-id", default=None)
    sub.add_parser("shutdown")
    a = ap.parse_args(argv)
    from moose_amd.cli.common import read_computation
    from moose_amd.runtime.choreography import ChoreographyClient
    from moose_amd.runtime.choreography import parse_session_file

    c = ChoreographyClient(a.store, a.timeout)
    if a.cmd == "shutdown":
        c.shutdown()
        return 0
    s = parse_session_file(a.session)
    sid = a.session_id or s["session_id"] or uuid.uuid4().hex
    idents = c.worker_identities(a.world)
    if a.cmd in ("launch", "run"):
        comp = read_computation(s["computation_path"], s["format"])
        ra = {role: (ep if ep in idents else role) for role, ep in s["roles"].items()}
        c.launch_computation(sid, comp, {}, ra)
        print(f"launched session {sid}")
    if a.cmd == "abort":
        c.abort_computation(sid)
        return 0
    if a.cmd in ("results", "run"):
        outs, timings = c.retrieve_results(sid, idents)
        for k in sorted(outs):
            print(f"{k} = {np.array2string(np.asarray(outs[k]), threshold=20)}")
        print(f"elapsed_us = {timings}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
