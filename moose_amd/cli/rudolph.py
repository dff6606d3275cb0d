"""``rudolph``: a party worker driven by the filesystem choreography.

Parity: reference ``moose/src/bin/rudolph/main.rs:12-97`` -- a worker that watches a
sessions directory for ``<session-id>.session`` TOML files (``[computation] path,
format`` + ``[[roles]] name, endpoint``) and runs each one once.  Here it is ``comet``
with the sessions watcher mandatory: rank 0 watches the directory and launches every new
file through the control-plane store; all ranks execute their share of the session::

    RANK=0 WORLD_SIZE=3 rudolph --identity alice --sessions ./sessions --store 127.0.0.1:29600
    RANK=1 WORLD_SIZE=3 rudolph --identity bob   --sessions ./sessions --store 127.0.0.1:29600
    RANK=2 WORLD_SIZE=3 rudolph --identity carole --sessions ./sessions --store 127.0.0.1:29600
"""
from __future__ import annotations

import argparse
import os
import sys

from moose_amd.cli import comet


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="rudolph", description=__doc__.splitlines()[0])
    ap.add_argument("--identity", required=True)
    ap.add_argument("--sessions", required=True, help="directory of *.session files")
    ap.add_argument("--store", default=os.environ.get("MOOSEX_STORE", "127.0.0.1:29600"))
    ap.add_argument("--backend", default=None)
    ap.add_argument("--storage-dir", default=None)
    ap.add_argument("--max-sessions", type=int, default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--ignore-existing", action="store_true",
                    help="ignore sessions already in the directory; only run new ones")
    ap.add_argument("--no-listen", action="store_true",
                    help="exit once the existing sessions have been processed")
    ap.add_argument("--telemetry", default=None, metavar="TRACE_JSON")
    a = ap.parse_args(argv)
    args = ["--identity", a.identity, "--store", a.store, "--sessions-dir", a.sessions]
    if a.port is not None:
        args += ["--port", str(a.port)]
    if a.ignore_existing:
        args.append("--ignore-existing")
    if a.no_listen:
        args.append("--no-listen")
    if a.telemetry:
        args += ["--telemetry", a.telemetry]
    if a.backend:
        args += ["--backend", a.backend]
    if a.storage_dir:
        args += ["--storage-dir", a.storage_dir]
    if a.max_sessions is not None:
        args += ["--max-sessions", str(a.max_sessions)]
    return comet.main(args)


if __name__ == "__main__":
    sys.exit(main())
