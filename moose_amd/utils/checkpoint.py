"""Per-party share checkpoints on disk (SURVEY §5 "checkpoint / resume").

The reference persists only Save/Load values and compiled computations
(``storage/filesystem/*``, ``computation.rs:1856-1874``).  Here a replicated ``Save``
(see :mod:`moose_amd.runtime.shares`) leaves every party's own pair of shares in that
party's storage; this module writes one party's storage to ``<dir>/<role>/`` and reads
it back, so each party persists only what it holds (no share ever leaves its owner).

Layout: a storage key ``a/b/c`` becomes ``<dir>/<role>/a/b/c.npy`` for arrays and
``.../c.json`` for strings/scalars.  Arrays are written and read with
``allow_pickle=False``.
"""
from __future__ import annotations

import json
import os
from typing import Dict
from typing import Iterable
from typing import Optional

import numpy as np


def _key_path(root: str, key: str) -> str:
    parts = [p for p in key.split("/") if p not in ("", ".", "..")]
    if not parts:
        raise ValueError(f"bad storage key {key!r}")
    return os.path.join(root, *parts)


def save_party(storage: Dict[str, object], directory: str, role: str,
               prefixes: Optional[Iterable[str]] = None) -> int:
    """Write one party's storage entries (optionally only keys under ``prefixes``)."""
    root = os.path.join(directory, role)
    n = 0
    for key, value in storage.items():
        if prefixes is not None and not any(key == p or key.startswith(p + "/")
                                            for p in prefixes):
            continue
        path = _key_path(root, key)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        if isinstance(value, (str, int, float, bool)) or value is None:
            with open(path + ".json", "w") as f:
                json.dump(value, f)
        else:
            np.save(path + ".npy", np.asarray(value), allow_pickle=False)
        n += 1
    return n


def load_party(directory: str, role: str) -> Dict[str, object]:
    """Read back everything :func:`save_party` wrote for ``role``."""
    root = os.path.join(directory, role)
    out: Dict[str, object] = {}
    for dirpath, _, files in os.walk(root):
        for fn in files:
            full = os.path.join(dirpath, fn)
            rel = os.path.relpath(full, root).replace(os.sep, "/")
            if fn.endswith(".npy"):
                out[rel[:-4]] = np.load(full, allow_pickle=False)
            elif fn.endswith(".json"):
                with open(full) as f:
                    out[rel[:-5]] = json.load(f)
    return out


def save_all(storages: Dict[str, Dict[str, object]], directory: str,
             prefixes: Optional[Iterable[str]] = None) -> int:
    """Simulation helper (``LocalMooseRuntime.storage``): every party's directory."""
    return sum(save_party(s, directory, role, prefixes) for role, s in storages.items())


def load_all(directory: str) -> Dict[str, Dict[str, object]]:
    return {role: load_party(directory, role) for role in sorted(os.listdir(directory))
            if os.path.isdir(os.path.join(directory, role))}
