"""ctypes binding of libaerognn.so (C-ABI declared in include/aerognn.h).

This is the drop-in boundary: every hot-path op of the reference's models/*.py is a call
through these entry points. There is deliberately NO fallback: if the shared library is
missing or a call fails, we raise.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# AEROGNN_LIB: an alternative build of the same library (A/B measurements only)
LIB_PATH = os.environ.get("AEROGNN_LIB") or os.path.join(_HERE, "libaerognn.so")

MAX_LIN = 8
MAX_SEG = 3
F32, BF16, F16, F64 = 0, 1, 2, 3
SEG_PLAIN, SEG_GATHER, SEG_SUM, SEG_MEAN = 0, 1, 2, 3
OPT_RESIDENT = 0

vp = C.c_void_p
i32 = C.c_int


class Seg(C.Structure):
    _fields_ = [("kind", i32), ("k", i32), ("ld", i32), ("_pad", i32),
                ("ptr", vp), ("index", vp), ("store", vp)]


# AGN_ACT_* (aerognn.h): the MLP hidden activation, mlp.py:37
ACT = {"relu": 0, "gelu": 1, "silu": 2, "tanh": 3}


class MlpFwdArgs(C.Structure):
    _fields_ = [("rows", i32), ("dtype", i32), ("hidden", i32), ("nlin", i32),
                ("out_dim", i32), ("nseg", i32), ("use_ln", i32), ("out_ld", i32),
                ("seg", Seg * MAX_SEG),
                ("wpk", vp * MAX_LIN), ("bias", vp * MAX_LIN),
                ("ln_g", vp), ("ln_b", vp),
                ("proj", vp), ("src", vp), ("dst", vp),
                ("resid", vp), ("out", vp),
                ("act", vp * MAX_LIN), ("hpre", vp), ("stats", vp), ("tiled", i32), ("act_fn", i32),
                ("mask", vp * MAX_LIN), ("pre", vp * MAX_LIN)]


class MlpBwdArgs(C.Structure):
    _fields_ = [("rows", i32), ("dtype", i32), ("hidden", i32), ("nlin", i32),
                ("out_dim", i32), ("in_dim", i32), ("use_ln", i32), ("ln_rows", i32),
                ("wtpk", vp * MAX_LIN), ("act", vp * MAX_LIN),
                ("hpre", vp), ("stats", vp), ("ln_g", vp),
                ("g", vp), ("g2", vp), ("gidx", vp),
                ("gpre", vp * MAX_LIN),
                ("din_nseg", i32), ("din_k", i32 * MAX_SEG),
                ("din", vp * MAX_SEG), ("din_resid", i32 * MAX_SEG),
                ("ln_partial", vp), ("tiled", i32), ("gpre_tiled", i32),
                ("mask", vp * MAX_LIN), ("act_fn", i32), ("_pad3", i32), ("pre", vp * MAX_LIN)]


MAX_WGRAD = 8


class WgradDesc(C.Structure):
    _fields_ = [("g", vp), ("x", vp), ("ldg", i32), ("ldx", i32), ("m", i32), ("k", i32), ("rows", i32),
                ("ldw", i32), ("dw_partial", vp), ("db_partial", vp), ("dw", vp), ("db", vp),
                ("g_tiled", i32), ("x_tiled", i32), ("nsplit", i32), ("_pad", i32), ("xidx", vp)]


class WgradBatch(C.Structure):
    _fields_ = [("n", i32), ("_pad", i32), ("d", WgradDesc * MAX_WGRAD)]


class WecArgs(C.Structure):
    _fields_ = [("n", i32), ("e", i32), ("dtype", i32), ("out_dim", i32), ("hid", i32), ("pos_dim", i32),
                ("pos_ld", i32), ("mean", i32),
                ("rowptr", vp), ("src", vp), ("dst", vp), ("perm", vp), ("rowptr_src", vp), ("perm_src", vp),
                ("pos", vp), ("pab", vp), ("tx", vp), ("w1c", vp), ("w2", vp),
                ("w_in", vp), ("w_out", vp), ("out", vp), ("dout", vp), ("gw", vp), ("s_csc", vp), ("dh", vp),
                ("dpa", vp), ("dpb", vp), ("dtx", vp), ("dw_in", vp), ("partial", vp)]


class EdgeBwdArgs(C.Structure):
    _fields_ = [("rows", i32), ("nblk", i32), ("wpk", vp * 4), ("bias", vp * 4), ("ln_g", vp), ("e", vp),
                ("proj", vp), ("src", vp), ("dst", vp), ("g", vp), ("g2", vp), ("de", vp), ("g0", vp),
                ("dw_partial", vp), ("db_partial", vp), ("ln_partial", vp), ("stamps", vp),
                ("a1", vp), ("stats", vp), ("scratch", vp), ("wtpk0", vp),
                ("xk", i32), ("xld", i32)]


class EdgeFwdArgs(C.Structure):
    _fields_ = [("rows", i32), ("nblk", i32), ("wpk", vp * 4), ("bias", vp * 4), ("ln_g", vp), ("ln_b", vp),
                ("e", vp), ("proj", vp), ("src", vp), ("dst", vp), ("out", vp), ("act", vp * 3), ("hpre", vp),
                ("stats", vp)]


class PackDesc(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("src_dtype", i32), ("dst_dtype", i32),
                ("rows", i32), ("cols", i32), ("trans", i32), ("ld", i32),
                ("row_off", i32), ("col_off", i32), ("dst_rows", i32), ("dst_cols", i32)]


class F64Seg(C.Structure):
    _fields_ = [("a", vp), ("aidx", vp), ("lda", i32), ("k", i32), ("w", vp), ("ldw", i32), ("transw", i32)]


class F64GemmArgs(C.Structure):
    _fields_ = [("rows", i32), ("n", i32), ("nseg", i32), ("_pad", i32), ("seg", F64Seg * 3), ("bias", vp),
                ("add", vp * 2), ("add_idx", vp * 2), ("add_ld", i32 * 2), ("mask", vp), ("mask_ld", i32),
                ("relu", i32), ("out", vp), ("out_ld", i32), ("mask_act", i32), ("pre_out", vp),
                ("pre_ld", i32), ("_pad3", i32)]


class F64WgradArgs(C.Structure):
    _fields_ = [("rows", i32), ("m", i32), ("k", i32), ("_pad", i32), ("g", vp), ("ldg", i32), ("_pad1", i32),
                ("x", vp), ("ldx", i32), ("_pad2", i32), ("xidx", vp), ("dw", vp), ("ldw", i32), ("_pad3", i32),
                ("db", vp)]


_lib = None

# Entry points that enqueue device work on a stream. When core.PROF is a list, every call of one
# of them is bracketed by HIP events on the caller's current stream (the stream the launch goes
# to) and recorded under its name, unless an enclosing core.timed(...) already times it under a
# finer tag (edge_fwd, node_bwd, ...). Nothing is recorded when PROF is None.
LAUNCHES = ("agn_pack", "agn_mlp_forward", "agn_mlp_backward", "agn_reduce_partials", "agn_wgrad", "agn_colsum",
            "agn_segment_sum", "agn_segment_sum2", "agn_gather_rows", "agn_radix_sort_u64", "agn_row_ptr", "agn_row_ptr_i64",
            "agn_iota_keys", "agn_level_index",
            "agn_exclusive_scan_i32", "agn_pool_sort_keys", "agn_pool_assign", "agn_pool_edge_candidates",
            "agn_pool_edge_sort", "agn_pool_edge_emit", "agn_bfs_distance", "agn_center_seed", "agn_maxdeg_seed",
            "agn_bistride_select", "agn_index_map", "agn_subgraph_edges", "agn_scatter_rows", "agn_wec_forward",
            "agn_wec_backward", "agn_edge_features", "agn_node_features", "agn_normalize", "agn_col_stats", "agn_collate",
            "agn_segment_max", "agn_segment_max_backward", "agn_edge_bwd_fused", "agn_encoder_bwd_fused", "agn_wgrad_reduce",
            "agn_edge_forward32",
            "agn_proj_forward", "agn_proj_backward")


class AeroGNNError(RuntimeError):
    pass


class _Lib:
    """The loaded CDLL; launch entry points go through the optional event timer."""

    def __init__(self, cdll):
        self._cdll = cdll
        for name in LAUNCHES:
            if hasattr(cdll, name):
                setattr(self, name, _timed_launch(getattr(cdll, name), name[4:]))

    def __getattr__(self, name):
        return getattr(self._cdll, name)


def _timed_launch(f, tag):
    from . import core

    def call(*args):
        prof = core.PROF
        if prof is None or core._TIMED_DEPTH:
            return f(*args)
        import torch
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        rc = f(*args)
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        prof.append((tag, None, s, e))
        return rc
    return call


def lib():
    """Load libaerognn.so (raises if it has not been built: no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AeroGNNError(
                f"{LIB_PATH} not found: build it with `make -C aero-gnn_amd/csrc` "
                "(or __graft_entry__.build()); the aerognn hot path has no CPU fallback")
        L = C.CDLL(LIB_PATH)
        sig = {
            "agn_version": (i32, []),
            "agn_error_string": (C.c_char_p, [i32]),
            "agn_set_option": (i32, [i32, i32]),
            "agn_packed_bytes": (C.c_size_t, [i32, i32, i32]),
            "agn_pack": (i32, [vp, i32, i32, vp]),
            "agn_mlp_forward": (i32, [C.POINTER(MlpFwdArgs), vp]),
            "agn_mlp_bwd_nwaves": (i32, [i32]),
            "agn_mlp_backward": (i32, [C.POINTER(MlpBwdArgs), vp]),
            "agn_reduce_partials": (i32, [vp, i32, i32, vp, vp]),
            "agn_wgrad_nsplit": (i32, [i32, i32]),
            "agn_wgrad_partial_floats": (C.c_size_t, [i32, i32, i32]),
            "agn_wgrad": (i32, [C.POINTER(WgradBatch), i32, i32, vp]),
            "agn_wgrad_plan": (i32, [C.POINTER(WgradBatch)]),
            "agn_colsum": (i32, [vp, i32, i32, vp, i32, vp, vp]),
            "agn_segment_sum": (i32, [i32, i32, i32, vp, vp, vp, i32, vp, i32, i32, vp]),
            "agn_segment_sum2": (i32, [i32, i32, i32, vp, i32, vp, vp, vp, i32, vp, vp, vp, i32, vp, i32, vp]),
            "agn_gather_rows": (i32, [i32, i32, i32, vp, vp, i32, vp, vp, i32, vp, i32, vp]),
            "agn_segment_max": (i32, [i32, i32, i32, vp, vp, vp, i32, vp, i32, vp, vp]),
            "agn_segment_max_backward": (i32, [i32, i32, i32, vp, vp, i32, vp, i32, vp]),
            "agn_radix_sort_temp_bytes": (C.c_size_t, [i32]),
            "agn_radix_sort_u64": (i32, [vp, vp, i32, i32, vp, vp, vp, vp]),
            "agn_row_ptr": (i32, [vp, i32, i32, vp, vp]),
            "agn_row_ptr_i64": (i32, [vp, i32, i32, vp, vp]),
            "agn_iota_keys": (i32, [i32, vp, vp, vp, vp, vp]),
            "agn_level_index": (i32, [i32, vp, C.c_int64, vp, vp, vp, vp, vp, vp, vp]),
            "agn_scan_temp_bytes": (C.c_size_t, [i32]),
            "agn_exclusive_scan_i32": (i32, [vp, vp, i32, vp, vp, vp]),
            "agn_pool_sort_keys": (i32, [i32, vp, vp, i32, vp, vp, vp]),
            "agn_pool_assign": (i32, [i32, i32, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp]),
            "agn_pool_edge_candidates": (i32, [i32, vp, vp, vp, vp, vp]),
            "agn_pool_edge_sort": (i32, [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
            "agn_pool_edge_emit": (i32, [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp]),
            "agn_bfs_work_ints": (C.c_size_t, [i32]),
            "agn_bfs_distance": (i32, [vp, vp, i32, i32, vp, vp, C.POINTER(i32), vp]),
            "agn_center_seed": (i32, [vp, i32, i32, i32, vp, vp]),
            "agn_maxdeg_seed": (i32, [vp, i32, vp, vp]),
            "agn_compact_work_ints": (C.c_size_t, [i32]),
            "agn_bistride_select": (i32, [vp, i32, vp, C.POINTER(i32), vp, vp]),
            "agn_index_map": (i32, [vp, i32, i32, vp, vp]),
            "agn_subgraph_edges": (i32, [vp, vp, i32, vp, vp, vp, C.POINTER(i32), vp, vp]),
            "agn_scatter_rows": (i32, [i32, i32, i32, vp, vp, i32, vp, i32, vp]),
            "agn_wec_blocks": (i32, [i32]),
            "agn_edge_bwd_blocks": (i32, [i32]),
            "agn_edge_bwd_scratch_bytes": (C.c_size_t, [i32]),
            "agn_edge_features": (i32, [i32, C.c_int64, i32, vp, vp, i32, vp, vp, vp, vp, vp]),
            "agn_normalize": (i32, [i32, i32, vp, i32, vp, vp, vp, i32, i32, vp]),
            "agn_col_stats_temp_bytes": (C.c_size_t, [i32, i32]),
            "agn_col_stats": (i32, [i32, i32, vp, i32, vp, vp, C.c_float, vp, vp]),
            "agn_collate": (i32, [i32, C.c_int64, C.c_int64, vp, vp, vp, vp, vp]),
            "agn_edge_bwd_fused": (i32, [C.POINTER(EdgeBwdArgs), vp]),
            "agn_encoder_bwd_fused": (i32, [C.POINTER(EdgeBwdArgs), vp]),
            "agn_edge_fwd32_blocks": (i32, [i32]),
            "agn_edge_forward32": (i32, [C.POINTER(EdgeFwdArgs), vp]),
            "agn_debug_node32_launches": (C.c_long, []),
            "agn_debug_enc32_launches": (C.c_long, []),
            "agn_debug_dec32_launches": (C.c_long, []),
            "agn_debug_node32_bwd_launches": (C.c_long, []),
            "agn_debug_dec32_bwd_launches": (C.c_long, []),
            "agn_fault_status": (i32, [C.POINTER(i32), i32]),
            "agn_fault_status_async": (i32, [vp, vp]),
            "agn_debug_set_fault": (i32, [i32]),
            "agn_wgrad_reduce": (i32, [C.POINTER(WgradBatch), i32, vp]),
            "agn_proj_forward": (i32, [i32, vp, i32, vp, vp, vp, i32, vp]),
            "agn_proj_backward": (i32, [i32, vp, vp, i32, vp, vp, i32, vp]),
            "agn_wec_forward": (i32, [C.POINTER(WecArgs), vp]),
            "agn_wec_backward": (i32, [C.POINTER(WecArgs), vp]),
            "agn_f64_gemm": (i32, [C.POINTER(F64GemmArgs), vp]),
            "agn_f64_wgrad_scratch_bytes": (C.c_size_t, [C.POINTER(F64WgradArgs)]),
            "agn_f64_wgrad": (i32, [C.POINTER(F64WgradArgs), vp, vp]),
            "agn_f64_layernorm_fwd": (i32, [i32, i32, vp, i32, vp, vp, vp, i32, vp, i32, vp, vp, C.c_double, vp]),
            "agn_f64_layernorm_bwd_scratch_bytes": (C.c_size_t, [i32, i32]),
            "agn_f64_layernorm_bwd": (i32, [i32, i32, vp, i32, vp, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp]),
        }
        for name, (res, args) in sig.items():
            if os.environ.get("AEROGNN_LIB") and name.startswith("agn_debug_") and not hasattr(L, name):
                continue  # an older A/B build without a newer kernel's debug counter
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = _Lib(L)
    return _lib


def exported_symbols():
    """Names of every function include/aerognn.h declares (checked by the CPU test suite)."""
    import re
    hdr = os.path.join(_HERE, "..", "..", "include", "aerognn.h")
    txt = open(hdr).read()
    return sorted(set(re.findall(r"\b(agn_[a-z0-9_]+)\s*\(", txt)))


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().agn_error_string(rc).decode()
        raise AeroGNNError(f"aerognn {what} failed: {msg} (code {rc})")


def fault_status(reset=True) -> int:
    """The device fault word (include/aerognn.h agn_fault_status): nonzero if a bounded LDS-ring
    wait of agn_edge_bwd_fused gave up since the last reset. Synchronises the device."""
    v = i32(0)
    check(lib().agn_fault_status(C.byref(v), 1 if reset else 0), "fault_status")
    return int(v.value)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()
