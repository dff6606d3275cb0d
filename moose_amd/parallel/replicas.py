"""Data-parallel replicas of a 3-party session (SURVEY §2.7 "DP": new, not in the
reference).

R replicas of an n-party session run on R disjoint groups of n GPUs (global rank =
``replica * n + party``).  Batch-shaped arguments are split along axis 0 across the
replicas; inside a replica every protocol message stays on that replica's process
group (RCCL point-to-point over xGMI); at the end the revealed outputs of the R replicas
are concatenated along axis 0 with ONE RCCL all-gather per output among the R ranks
that own it (a direct-link collective: with R <= 3 every pair of owners has its own
xGMI link).
"""
from __future__ import annotations

from typing import Dict
from typing import Iterable
from typing import List

import numpy as np
import torch


def shard_arguments(arguments: dict, names: Iterable[str], replicas: int) -> List[dict]:
    """Per-replica argument dicts: ``names`` split along axis 0 (np.array_split: the
    first ``len % R`` replicas get one extra row), everything else replicated."""
    names = set(names or ())
    missing = names - set(arguments)
    if missing:
        raise KeyError(f"shard_args names unknown arguments: {sorted(missing)}")
    out = [dict() for _ in range(replicas)]
    for k, v in arguments.items():
        if k in names:
            a = np.asarray(v)
            if a.ndim == 0 or a.shape[0] < replicas:
                raise ValueError(f"argument {k!r} with shape {a.shape} cannot be split "
                                 f"across {replicas} replicas")
            for r, part in enumerate(np.array_split(a, replicas, axis=0)):
                out[r][k] = np.ascontiguousarray(part)
        else:
            for r in range(replicas):
                out[r][k] = v
    return out


def make_groups(n_parties: int, replicas: int):
    """(replica groups, owner groups): every rank must call this, in the same order.
    ``replica_groups[r]`` = the n ranks of replica r; ``owner_groups[p]`` = party p of
    every replica."""
    import torch.distributed as dist

    rg = [dist.new_group([r * n_parties + p for p in range(n_parties)])
          for r in range(replicas)]
    og = [dist.new_group([r * n_parties + p for r in range(replicas)])
          for p in range(n_parties)]
    return rg, og


def gather_rows(a: np.ndarray, group, replicas: int, device) -> np.ndarray:
    """Concatenate ``a`` of every replica along axis 0 (ragged first dim allowed)."""
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(a.view(np.int64) if a.dtype == np.uint64
                                              else a.astype(np.uint8) if a.dtype == bool
                                              else a)).to(device)
    rows = torch.tensor([t.shape[0]], dtype=torch.int64, device=device)
    all_rows = torch.empty(replicas, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(all_rows, rows, group=group)
    counts = [int(c) for c in all_rows.cpu()]
    mx = max(counts)
    if t.shape[0] < mx:
        pad = torch.zeros((mx - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=device)
        t = torch.cat([t, pad])
    buf = torch.empty((replicas * mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=device)
    dist.all_gather_into_tensor(buf, t.contiguous(), group=group)
    parts = [buf[r * mx: r * mx + c] for r, c in enumerate(counts)]
    out = torch.cat(parts).cpu().numpy()
    if a.dtype == np.uint64:
        return out.view(np.uint64)
    if a.dtype == bool:
        return out.astype(bool)
    return out


def gather_outputs(outs: Dict[str, object], group, replicas: int, device) -> Dict[str, object]:
    """All-gather every numeric output with a leading axis across the replicas' owners
    (same tag order on every owner rank); other outputs keep replica 0's value."""
    res = {}
    for tag in sorted(outs):
        v = outs[tag]
        a = np.asarray(v) if not isinstance(v, (str, bytes)) else None
        if a is not None and a.ndim >= 1 and a.dtype.kind in "biuf":
            res[tag] = gather_rows(a, group, replicas, device)
        else:
            res[tag] = v
    return res
