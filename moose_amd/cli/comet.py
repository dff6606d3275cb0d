"""``comet``: a party worker serving choreographed sessions.

Parity: reference ``moose/src/bin/comet/comet.rs:12-83`` (flags ``--identity``,
``--port``; gRPC choreography + networking + filesystem storage).  Here one worker per
identity joins a process group whose rank 0 hosts the control-plane store::

    RANK=0 WORLD_SIZE=3 comet --identity alice --store 127.0.0.1:29600 --backend nccl
    RANK=1 WORLD_SIZE=3 comet --identity bob   --store 127.0.0.1:29600 --backend nccl
    ...

``--sessions-dir`` additionally watches a directory of ``.session`` files on rank 0
(the reference's ``rudolph`` filesystem choreography).
"""
from __future__ import annotations

import argparse
import os
import sys
import threading


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="comet", description=__doc__.splitlines()[0])
    ap.add_argument("--identity", required=True)
    ap.add_argument("--store", default=os.environ.get("MOOSEX_STORE", "127.0.0.1:29600"))
    ap.add_argument("--rank", type=int, default=int(os.environ.get("RANK", 0)))
    ap.add_argument("--world", type=int, default=int(os.environ.get("WORLD_SIZE", 3)))
    ap.add_argument("--backend", default=None, help="nccl (RCCL, one GPU per worker) | gloo")
    ap.add_argument("--storage-dir", default=None, help="filesystem storage (*.npy)")
    ap.add_argument("--sessions-dir", default=None, help="watch *.session files (rank 0)")
    ap.add_argument("--max-sessions", type=int, default=None)
    ap.add_argument("--port", type=int, default=None,
                    help="control-plane port (overrides the port of --store)")
    ap.add_argument("--telemetry", default=None, metavar="TRACE_JSON",
                    help="write a Chrome trace of this worker's spans ({identity} expands)")
    ap.add_argument("--ignore-existing", action="store_true",
                    help="with --sessions-dir: only sessions that appear after start-up")
    ap.add_argument("--no-listen", action="store_true",
                    help="with --sessions-dir: run the existing sessions, then shut down")
    a = ap.parse_args(argv)
    if a.port is not None:
        a.store = f"{a.store.rsplit(':', 1)[0]}:{a.port}"
    if a.telemetry:
        from moose_amd.utils.telemetry import enable_tracing

        enable_tracing(a.telemetry.replace("{identity}", a.identity))
    import torch

    from moose_amd.runtime.choreography import ChoreographyClient
    from moose_amd.runtime.choreography import Worker
    from moose_amd.runtime.choreography import watch_sessions

    backend = a.backend or ("nccl" if torch.cuda.device_count() >= a.world else "gloo")
    w = Worker(a.identity, a.rank, a.world, a.store, backend, a.storage_dir)
    stop = threading.Event()
    th = None
    if a.sessions_dir and a.rank == 0:
        client = ChoreographyClient(a.store)
        th = threading.Thread(target=watch_sessions,
                              args=(a.sessions_dir, client, a.world, stop),
                              kwargs={"ignore_existing": a.ignore_existing,
                                      "no_listen": a.no_listen}, daemon=True)
        th.start()
    try:
        return w.serve(a.max_sessions)
    finally:
        stop.set()


if __name__ == "__main__":
    sys.exit(main())
