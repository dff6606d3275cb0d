"""Session PRF keys held in device memory ("key slots").

Every PRF evaluation of a session -- zero shares, input sharing, the dealer masks of
TruncPr, seeded sampling -- is a ChaCha12 keystream (``csrc/prf_core.h``) under one of the
session's keys.  Instead of passing keys as launch parameters, the session keeps them in a
:class:`KeyTable`: one device tensor of ``MX_KEY_SLOT_WORDS``-word slots (the raw 128-bit key
in words 0..3, followed by its AES-128 schedule for the AES dialect, ``csrc/moosex.h``) that
the kernels read at run time.  Two things follow:

* a hipGraph captured from an evaluation does not bake the keys in: refreshing the table
  before each replay gives every replay fresh, independent randomness
  (:mod:`moose_amd.runtime.graphs`);
* setup costs one small host->device copy per placement instead of a key expansion per
  kernel launch.

Parity: the keys play the role of the reference's ``RepSetup`` PRF keys
(``replicated/setup.rs:39-58``) and the seeds of ``PrfKeyGen``/``DeriveSeed``
(``host/prim.rs:113-150``).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from moose_amd.ops import native as nat

SLOT_WORDS = 48  # MX_KEY_SLOT_WORDS
_PINNED = os.environ.get("MOOSEX_KEYS_PINNED", "1") != "0"


class KeyRef:
    """A seed that lives in a key slot (what ``h_fresh_seed`` hands out)."""

    __slots__ = ("table", "slot")

    def __init__(self, table: "KeyTable", slot: int):
        self.table = table
        self.slot = slot

    @property
    def ptr(self):
        return self.table.ptr(self.slot)

    def __len__(self):
        return 16


class KeyBuf:
    """A fresh seed received from its owner: the owner's key slot image (raw key and AES
    schedule, SLOT_WORDS int32) in a buffer of the receiver (parallel/spmd.py move).  Like
    :class:`KeyRef`, SampleSeeded expands it from ``ptr``."""

    __slots__ = ("t",)
    table = None  # SampleSeeded tells key-slot seeds from raw bytes by this attribute

    def __init__(self, t: torch.Tensor):
        self.t = t

    @property
    def ptr(self):
        return self.t.data_ptr()

    def __len__(self):
        return 16


def slot_words(keys) -> np.ndarray:
    """Host image of ``len(keys)`` slots."""
    raw = b"".join(bytes(k) for k in keys)
    out = np.zeros((len(keys), SLOT_WORDS), dtype=np.uint32)
    nat.lib().mx_key_slots(ctypes.c_char_p(raw), len(keys),
                           out.ctypes.data_as(ctypes.c_void_p))
    return out


def _lanes_active(device) -> bool:
    from moose_amd.runtime import lanes

    return lanes.ACTIVE and device.type == "cuda"


class KeyTable:
    """Fixed-capacity table of key slots on ``device``.

    ``alloc`` hands out consecutive slots and (unless the table is *frozen*) fills them
    with fresh keys.  A frozen table -- the state during hipGraph capture -- never writes:
    its contents were filled by :meth:`refresh` beforehand and are refreshed again before
    each replay.
    """

    def __init__(self, device, capacity: int = 256, random_bytes=None):
        self.device = torch.device(device)
        self.capacity = capacity
        self.t = torch.zeros((capacity, SLOT_WORDS), dtype=torch.int32, device=self.device)
        self.n = 0
        self.frozen = False
        self._rand = random_bytes or os.urandom
        self.allocs = []  # (base, n) of the allocations made while frozen, in order

    def alloc(self, n: int) -> int:
        base = self.n
        if base + n > self.capacity:
            if self.frozen:
                raise RuntimeError("key table exhausted during graph capture")
            if _lanes_active(self.device):  # kernels on other lanes may still read self.t
                torch.cuda.synchronize(self.device)
            grown = torch.zeros((max(2 * self.capacity, base + n), SLOT_WORDS),
                                dtype=torch.int32, device=self.device)
            grown[:self.capacity].copy_(self.t)
            self.t, self.capacity = grown, grown.shape[0]
        self.n = base + n
        if not self.frozen:
            self._write(base, [self._rand(16) for _ in range(n)])
        else:
            self.allocs.append((base, n))  # a replay refills these slots (refresh_seeded)
        return base

    def _write(self, base: int, keys):
        img = torch.from_numpy(slot_words(keys).view(np.int32))
        if self.device.type == "cuda" and _PINNED:
            # a pinned staging copy + asynchronous DMA in stream order: a pageable copy
            # would block the host until the stream drained (a host sync per session
            # setup / per graph replay).  The caching host allocator keeps the staging
            # buffer alive until the copy has run.
            self.t[base:base + len(keys)].copy_(img.pin_memory(), non_blocking=True)
        else:
            self.t[base:base + len(keys)].copy_(img)
        if _lanes_active(self.device):  # readers on other streams see complete keys
            torch.cuda.current_stream(self.device).synchronize()

    def refresh(self, upto: int = None):
        """Fresh random keys for slots ``[0, upto)`` (default: every slot).  One urandom
        call for all of them (per-slot calls cost 0.23 ms per 256 slots on the host)."""
        n = self.capacity if upto is None else upto
        raw = os.urandom(16 * n)
        self._write(0, [raw[16 * i:16 * i + 16] for i in range(n)])

    def refresh_seeded(self, seed: int):
        """The keys a fresh session seeded with ``seed`` draws, in the slots its allocations
        get (the frozen table's recorded allocations): a replay of a seeded evaluation then
        uses exactly the eager evaluation's keys (bitwise-equal replays)."""
        rng = torch.Generator().manual_seed(seed)
        for base, n in self.allocs:
            self._write(base, [bytes(torch.randint(0, 256, (16,), generator=rng,
                                                   dtype=torch.uint8).tolist())
                               for _ in range(n)])

    def enable_device_refresh(self):
        """Draw the keys of later :meth:`refresh_device` calls on the device: a master key
        from the OS (16 bytes, uploaded once) and a replay counter in device memory
        (csrc/party_graph.hip ``mx_key_refresh``)."""
        raw = np.frombuffer(os.urandom(16), dtype=np.int32).copy()
        self._master = torch.from_numpy(raw).to(self.device)
        self._epoch = torch.zeros(1, dtype=torch.int64, device=self.device)

    def refresh_device(self, upto: int = None):
        """Fresh keys for slots ``[0, upto)`` drawn by ONE kernel on the current stream:
        slot s of the e-th refresh = ChaCha12(master, nonce e, block s)'s first 16 bytes and
        its AES-128 schedule.  No host work beyond the launch (a replay's key refresh was a
        urandom call, the schedules and a pinned copy per table on the host)."""
        n = self.capacity if upto is None else upto
        if self.device.type != "cuda" or getattr(self, "_master", None) is None:
            return self.refresh(n)
        nat.check(nat.lib().mx_key_refresh(self.t.data_ptr(), n, self._master.data_ptr(),
                                           self._epoch.data_ptr(), nat.stream_of(self.t)),
                  "key refresh")

    def ptr(self, slot: int) -> int:
        return self.t.data_ptr() + slot * SLOT_WORDS * 4

    def raw_key(self, slot: int) -> bytes:
        """The raw 16-byte key of a slot (reads device memory; host-side uses only)."""
        return self.t[slot, :4].cpu().numpy().astype(np.int32).tobytes()
