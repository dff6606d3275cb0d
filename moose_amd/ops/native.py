"""ctypes binding of the native core ``libmoosex.so`` (built in-tree on first use).

On a GPU box the device kernels are mandatory: if the library cannot be loaded we raise
instead of silently falling back to a slower path.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from moose_amd import errors
from moose_amd._native import build as _build

_LIB = None
_LOCK = threading.Lock()

c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_u64 = ctypes.c_uint64
c_vp = ctypes.c_void_p

_SIGS = {
    "mx_version": (c_int, []),
    "mx_device_count": (c_int, []),
    "mx_ew_binary": (c_int, [c_int, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mx_ew_unary": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "mx_mul_add2": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_int, c_int, c_vp, c_vp,
                            c_i64, c_vp]),
    "mx_ew_binary2": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                              c_i64, c_i64, c_vp]),
    "mx_ew_unary2": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "mx_transpose2": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    "mx_ew_binary_slot2": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp,
                                   c_i64, c_int, c_int, c_int, c_vp]),
    "mx_mul_trunc3_kv": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                 c_vp, c_u64, c_int, c_vp, c_vp, c_vp]),
    "mx_ew_add3": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mx_lincomb2": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64,
                            c_int, c_int, c_int, c_vp]),
    "mx_sum_views2": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_vp,
                              c_vp, c_i64, c_int, c_vp]),
    "mx_slot_place2": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_int,
                               c_vp]),
    "mx_ew_compare": (c_int, [c_int, c_int, c_int, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp]),
    "mx_bit_extract": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_int, c_vp]),
    "mx_ring_inject": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_int, c_vp]),
    "mx_encode": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_int, c_vp]),
    "mx_decode": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_int, c_vp]),
    "mx_addn_decode": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp]),
    "mx_sum_axis": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "mx_fill": (c_int, [c_int, c_int, c_vp, c_i64, c_u64, c_u64, c_vp]),
    "mx_bit_planes": (c_int, [c_int, c_int, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_vp]),
    "mx_weighted_sum": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp]),
    "mx_prg": (c_int, [c_int, c_vp, c_u64, c_u64, c_vp, c_i64, c_vp]),
    "mx_aes_encrypt_blocks": (c_int, [c_vp, c_vp, c_vp, c_i64]),
    "mx_derive_seed": (c_int, [c_vp, c_vp, c_vp]),
    "mx_rss_cross": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_u64, c_vp],
    ),
    "mx_zero_share": (c_int, [c_int, c_int, c_int, c_vp, c_i64, c_int, c_vp, c_u64, c_vp]),
    "mx_prf_expand": (c_int, [c_int, c_int, c_vp, c_i64, c_int, c_vp, c_u64, c_vp]),
    "mx_gemm": (
        c_int,
        [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp],
    ),
    "mx_gemm_workspace_bytes": (c_i64, [c_int, c_i64, c_i64, c_i64, c_i64, c_int]),
    "mx_workspace_failed_bytes": (c_i64, []),
    "mx_workspace_held_bytes": (c_i64, []),
    "mx_workspace_shared_count": (c_i64, []),
    "mx_mfma_peak": (c_int, [c_int, c_int, c_vp, c_vp]),
    "mx_gemm_ws": (
        c_int,
        [c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_int, c_vp,
         c_i64, c_vp],
    ),
    "mx_set_gemm_impl": (None, [c_int]),
    "mx_set_gemm_crt": (None, [c_int]),
    "mx_gemm_strided": (
        c_int,
        [c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_vp,
         c_int, c_vp],
    ),
    "mxh_wsum_trunc3": (
        c_int, [c_int, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp,
                c_vp, c_vp, c_vp],
    ),
    "mxh_mul_trunc3_kv2": (
        c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                c_vp, c_vp],
    ),
    "mxh_b2a_prep3": (c_int, [c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "mxh_b2a3_planes": (
        c_int, [c_int, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_u64, c_u64,
                c_vp],
    ),
    "mxh_mul_rows_add": (c_int, [c_int, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_int, c_int, c_vp]),
    "mxh_mux3": (
        c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_u64, c_int,
                c_vp],
    ),
    "mxh_bitdec3": (
        c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_u64, c_u64, c_vp,
                c_int, c_u64, c_u64, c_vp],
    ),
    "mxh_b2a3": (
        c_int, [c_int, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_int, c_u64, c_u64, c_vp],
    ),
    "mxh_gemm_bs": (
        c_int, [c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp],
    ),
    "mx_crt_moduli": (c_int, [c_int, c_i64]),
    "mx_crt_tables": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_trunc_pr3": (
        c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp],
    ),
    "mx_key_slots": (None, [ctypes.c_char_p, c_int, c_vp]),
    "mx_rss_cross_k": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_int, c_u64,
         c_vp],
    ),
    "mx_prf_expand_k": (c_int, [c_int, c_int, c_vp, c_i64, c_int, c_vp, c_u64, c_vp]),
    "mx_add_zs3": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    "mx_ew_binary_slot": (
        c_int, [c_int, c_int, c_int, c_vp, c_vp, c_i64, c_vp, c_i64, c_int, c_int, c_vp]),
    "mx_ks_cross1": (
        c_int,
        [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_u64, c_vp],
    ),
    "mx_ks_cross1_s": (
        c_int,
        [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_u64, c_vp],
    ),
    "mx_ks_cross1x_s": (
        c_int,
        [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int,
         c_vp, c_u64, c_vp],
    ),
    "mx_ks_sum2": (
        c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    ),
    "mx_ks_adder3_k": (
        c_int,
        [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp],
    ),
    "mxh_ks_adder3_sum": (
        c_int,
        [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_int],
    ),
    "mx_ks_level3_k": (
        c_int,
        [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_int,
         c_vp, c_u64, c_vp],
    ),
    "mx_rss_cross_kp": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_u64, c_vp],
    ),
    "mx_rss_mul3_kv": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_u64, c_vp, c_vp],
    ),
    "mx_rss_mul3_k": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_u64, c_vp],
    ),
    "mx_trunc_pr3_k": (
        c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_vp],
    ),
    "mx_trunc_pr3_ko": (
        c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp],
    ),
    "mx_trunc_pr3_kmo": (
        c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp, c_i64, c_vp,
                c_vp],
    ),
    "mx_share3_k": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_u64, c_u64, c_vp],
    ),
    "mx_trunc_party_r0": (
        c_int,
        [c_int, c_int, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
         c_vp, c_vp],
    ),
    "mx_trunc_party_r1": (
        c_int,
        [c_int, c_int, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
         c_vp, c_vp, c_vp],
    ),
    "mx_dot_tail_r0": (
        c_int,
        [c_int, c_int, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
         c_vp, c_vp],
    ),
    "mx_dot_tail_r1": (
        c_int,
        [c_int, c_int, c_i64, c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
         c_vp, c_vp, c_vp, c_vp],
    ),
    "mx_dot_tail_r2": (c_int, [c_int, c_int, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_share_party": (
        c_int,
        [c_int, c_int, c_int, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_u64, c_u64, c_vp],
    ),
    "mx_gemm_b_bytes": (c_i64, [c_int, c_i64, c_i64, c_i64, c_int]),
    "mx_gemm_prep_b": (c_int, [c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_int, c_vp, c_vp]),
    "mx_gemm_with_b": (
        c_int,
        [c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_int, c_vp],
    ),
    "mx_share3": (
        c_int,
        [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_u64, c_u64, c_vp],
    ),
    "mx_crt_tables4": (c_int, [c_int, c_int, c_vp, c_vp]),
    "mx_copy_channels": (c_int, [c_vp, c_vp, c_i64, c_int, c_vp]),
    "mx_stream_cumask": (c_int, [c_vp, c_int, c_vp]),
    "mx_stream_destroy": (c_int, [c_vp]),
    "mx_graph_compose": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    # (n, kind, child, dst, src, bytes, party, stats[4], graph*, exec*): party-batched chain
    "mx_graph_compose_merged": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                        c_vp]),
    "mx_graph_dot": (c_int, [c_vp, ctypes.c_char_p, ctypes.c_uint]),
    "mx_graph_launch": (c_int, [c_vp, c_vp]),
    "mx_enable_peer": (c_int, [c_int, c_int]),
    "mx_alloc_uncached": (c_int, [c_int, c_i64, c_vp]),
    "mx_free_uncached": (c_int, [c_int, c_vp]),
    "mx_graph_build_chain": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                     c_vp]),
    "mx_jobs_r0": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int,
                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_jobs_r0p": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int,
                            c_vp, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp, c_vp]),
    "mx_jobs_r1": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_vp,
                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_jobs_r2": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_i64, c_int, c_vp, c_vp, c_vp]),
    "mx_bits_front": (c_int, [c_int, c_int, c_int, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                              c_vp, c_vp, c_vp, c_vp]),
    "mx_wsum_pair": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_i64, c_i64,
                             c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_vp, c_vp, c_vp]),
    "mx_bits_b2a": (c_int, [c_int, c_int, c_int, c_int, c_i64, c_int, c_int, c_int, c_int,
                            c_vp, c_vp, c_vp,
                            c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "mx_key_refresh": (c_int, [c_vp, c_int, c_vp, c_vp, c_vp]),
    "mx_copy_async": (c_int, [c_vp, c_vp, ctypes.c_int64, c_vp]),
    "mx_key_refresh_host": (None, [c_vp, c_u64, c_int, c_vp]),
    "mx_copy_many": (c_int, [c_vp, c_int, c_i64, c_vp]),
    "mx_graph_free": (c_int, [c_vp, c_vp]),
    "mx_gemm_asym": (
        c_int, [c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int, c_vp, c_vp],
    ),
    "mx_gemm_roll": (
        c_int,
        [c_int, c_i64, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_int,
         c_vp],
    ),
}


class NativeError(errors.KernelError):
    pass


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if _build.needs_build() and os.environ.get("MOOSEX_NO_BUILD") != "1":
            _build.build()
        path = os.environ.get("MOOSEX_LIB") or str(_build.LIB)  # tuning variants
        try:
            handle = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:
            raise NativeError(f"cannot load {path}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
        return _LIB


def loaded_path():
    return str(_build.LIB)


def check(rc, what):
    if rc != 0:
        if rc == -4:
            raise NativeError(workspace_error(what, _ws_failed_bytes(), _ws_held_bytes()))
        raise NativeError(f"{what} failed with code {rc}")


def _ws_failed_bytes() -> int:
    try:
        return int(lib().mx_workspace_failed_bytes())
    except Exception:  # noqa: BLE001 - an older library: no size known
        return 0


def _ws_held_bytes() -> int:
    try:
        return int(lib().mx_workspace_held_bytes())
    except Exception:  # noqa: BLE001
        return 0


def workspace_error(what: str, failed: int, held: int) -> str:
    """Message of a GEMM whose device scratch could not be allocated (return code -4)."""
    gib = 1 << 30
    size = f"{failed / gib:.2f} GiB" if failed else "an unknown size"
    return (f"{what} failed with code -4: the device workspace allocation of {size} "
            f"({failed} bytes) failed; {held / gib:.2f} GiB of GEMM workspace already held on "
            "this device.  The scratch is grow-only per (device, stream) -- see docs/API.md "
            "'Device memory' for the per-stream footprint; use fewer step streams or "
            "processes per GPU, or smaller products")


def dev_of(t: torch.Tensor) -> int:
    return 1 if t.is_cuda else 0


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t: torch.Tensor):
    """The current HIP stream of t's device as a raw handle (None on the host).  This is
    on every launch's path, so it skips torch.cuda.current_stream's Stream object."""
    if t.is_cuda:
        if _raw_stream is not None:
            return _raw_stream(t.get_device())
        return torch.cuda.current_stream(t.device).cuda_stream
    return None


def ptr(t):
    # plain ints: the c_void_p argtypes convert them (no ctypes object per operand)
    return None if t is None else t.data_ptr()


def key_buffer(keys) -> ctypes.Array:
    """Pack a list of 16-byte keys into a C buffer."""
    raw = b"".join(bytes(k) for k in keys)
    return ctypes.create_string_buffer(raw, len(raw))


class _UncachedBlock:
    """``bytes`` of uncached device memory (mx_alloc_uncached), exposed to torch through
    ``__cuda_array_interface__``; freed when the last tensor viewing it is gone (torch keeps
    the exporting object alive for the storage's lifetime)."""

    def __init__(self, dev: int, nbytes: int):
        p = ctypes.c_void_p()
        check(lib().mx_alloc_uncached(dev, int(nbytes), ctypes.byref(p)),
              f"uncached device allocation of {nbytes} bytes")
        self.dev, self.ptr, self.nbytes = dev, p.value, int(nbytes)
        self.__cuda_array_interface__ = {"shape": (self.nbytes,), "typestr": "|u1",
                                         "data": (self.ptr, False), "version": 2,
                                         "strides": None}

    def __del__(self):
        try:
            if self.ptr:
                lib().mx_free_uncached(self.dev, ctypes.c_void_p(self.ptr))
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def uncached_zeros(shape, dtype, device) -> torch.Tensor:
    """A zero-filled tensor in uncached device memory (csrc/party_graph.hip
    mx_alloc_uncached): what a PEER GPU writes while this one polls or later reads it --
    message flags and landing buffers of the per-party stream graphs (threads.py)."""
    import math

    device = torch.device(device)
    el = torch.empty((), dtype=dtype).element_size()
    n = math.prod(shape) if len(shape) else 1
    blk = _UncachedBlock(device.index if device.index is not None else 0, max(1, n) * el)
    with torch.cuda.device(device):
        raw = torch.as_tensor(blk, device=device)
    return raw[:n * el].view(dtype).reshape(tuple(shape))
