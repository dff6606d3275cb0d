"""Storage backends: in-memory dicts and filesystem (``.npy`` / ``.csv``).

Parity: reference ``moose/src/storage/{local,filesystem/{csv,numpy}}.rs`` -- the key is
a file path; ``.csv`` loads accept a JSON query ``{"select_columns": [...]}``; ``.npy``
dtype comes from the file header.  Loading uses ``numpy.load(allow_pickle=False)``.
"""
from __future__ import annotations

import csv
import json
import os
from typing import Any
from typing import Dict

import numpy as np


def looks_like_path(key: str) -> bool:
    return isinstance(key, str) and (key.endswith(".npy") or key.endswith(".csv"))


def load_from_path(path: str, query: str = "") -> Any:
    if not os.path.exists(path):
        return None
    if path.endswith(".npy"):
        return np.load(path, allow_pickle=False)
    if path.endswith(".csv"):
        cols = None
        if query:
            q = json.loads(query)
            cols = q.get("select_columns")
        with open(path, newline="") as f:
            rows = list(csv.reader(f))
        header, body = rows[0], rows[1:]
        idx = list(range(len(header))) if cols is None else [header.index(c) for c in cols]
        return np.array([[float(r[i]) for i in idx] for r in body], dtype=np.float64)
    raise ValueError(f"unsupported storage path {path}")


def save_to_path(path: str, value) -> None:
    value = np.asarray(value)
    if path.endswith(".npy"):
        np.save(path, value, allow_pickle=False)
    elif path.endswith(".csv"):
        v = np.atleast_2d(value)
        with open(path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow([f"column_{i}" for i in range(v.shape[1])])
            for row in v:
                w.writerow([repr(float(x)) for x in row])
    else:
        raise ValueError(f"unsupported storage path {path}")


class LocalStorage:
    """In-memory key/value storage of one identity (reference storage/local.rs)."""

    def __init__(self, initial: Dict[str, Any] = None):
        self.data = dict(initial or {})

    def save(self, key, value):
        self.data[key] = value

    def load(self, key, query=""):
        if key in self.data:
            return self.data[key]
        if looks_like_path(key):
            v = load_from_path(key, query)
            if v is not None:
                return v
        raise KeyError(key)


class FilesystemStorage(LocalStorage):
    """Keys are file paths (reference storage/filesystem/mod.rs:16-88)."""

    def save(self, key, value):
        if looks_like_path(key):
            save_to_path(key, value)
        else:
            super().save(key, value)
