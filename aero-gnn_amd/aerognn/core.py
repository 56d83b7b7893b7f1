"""Thin host wrappers over the C-ABI (launch arguments, workspaces, weight packing).

Everything here runs on the caller's current HIP stream; nothing synchronises.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from ._lib import check, ptr


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


# --------------------------------------------------------------------------- launch timing
# When PROF is a list, every tagged kernel launch is bracketed by HIP events recorded on the
# stream it runs on (torch's current stream): entries (tag, (alg_bytes, alg_flops), start, end).
# Untagged launches are recorded under their entry-point name by _lib (see _lib.LAUNCHES).
PROF = None
_TIMED_DEPTH = 0


class _Timed:
    __slots__ = ("tag", "cost", "s", "on")

    def __init__(self, tag, cost):
        self.tag, self.cost = tag, cost
        self.on = False

    def __enter__(self):
        global _TIMED_DEPTH
        if PROF is not None and self.tag is not None:
            self.on = True
            _TIMED_DEPTH += 1
            self.s = torch.cuda.Event(enable_timing=True)
            self.s.record()
        return self

    def __exit__(self, *a):
        global _TIMED_DEPTH
        if self.on:
            _TIMED_DEPTH -= 1
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            if PROF is not None:
                PROF.append((self.tag, self.cost, self.s, e))
        return False


def timed(tag, cost=None):
    return _Timed(tag, cost)


def dt_code(dtype) -> int:
    if dtype == torch.float32:
        return L.F32
    if dtype == torch.bfloat16:
        return L.BF16
    if dtype == torch.float16:
        return L.F16
    if dtype == torch.float64:  # graph ops and the agn_f64_* kernels (aerognn/f64.py)
        return L.F64
    raise NotImplementedError(f"aerognn kernels compute in float64, float32, bfloat16 or float16, got {dtype}")


def tiled_empty(rows, width, dtype, device):
    """[rows, width] buffer in the AGN_TILED layout (aerognn.h): rows padded to 32, only
    libaerognn reads it. Tagged so mlp_forward / mlp_backward / WGrad pass the layout on."""
    t = torch.empty((rows + 31) // 32 * 32, width, dtype=dtype, device=device)
    t.agn_tiled = True
    t.agn_rows = rows
    return t


def relu_mask_empty(rows, width, device):
    """AGN_RELU_MASK buffer (aerognn.h) for a [rows, width] ReLU output: max(1, width / 64)
    dwords per lane of each 32-row tile."""
    nd = max(1, (width + 63) // 64)
    return torch.empty((rows + 31) // 32 * nd * 64, dtype=torch.int32, device=device)


def _mask_of(t):
    """The backward reads ReLU sign bits (AGN_RELU_MASK, attached to each saved activation by
    the allocator) instead of the activations, which are saved for agn_wgrad only."""
    return getattr(t, "agn_mask", None)


def _pre_of(t):
    """A non-ReLU activation's backward reads the saved pre-activation (attached by the allocator)."""
    return getattr(t, "agn_pre", None)


def is_tiled(t) -> bool:
    return t is not None and getattr(t, "agn_tiled", False)


def logical_rows(t) -> int:
    return getattr(t, "agn_rows", t.shape[0])


def require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("aerognn: tensors must live on the MI355X (HIP device); the hot path "
                               "has no CPU implementation (the CPU oracle is test-only)")


def packed_bytes(m, k, dtype_code):
    return int(L.lib().agn_packed_bytes(int(m), int(k), int(dtype_code)))


# ----------------------------------------------------------------------------- weight packing
class Pack:
    """Packed MFMA A-operands + fp32 parameter vectors of one module, in one workspace.

    `matrix(key, M, K, parts)`: parts = [(W, row_off, col_off, trans)], A[r][k] = W[r][k]
    (or W[k][r] when trans) placed at (row_off, col_off) of an [M x K] operand.
    `vector(key, n, parts)`: parts = [(v, off)] copied to fp32 (zeros elsewhere).
    Re-run `update()` every forward (weights change after each optimizer step): one launch.
    """

    def __init__(self):
        self.mats = {}
        self.vecs = {}
        self._sig = None
        self.ws = None
        self.views = {}
        self._descs = None

    def matrix(self, key, M, K, parts):
        self.mats[key] = (int(M), int(K), parts)

    def vector(self, key, n, parts):
        self.vecs[key] = (int(n), parts)

    def _signature(self, dtype):
        sig = [dtype]
        for key, (M, K, parts) in self.mats.items():
            sig += [(key, p[0].data_ptr(), p[0].dtype) for p in parts]
        for key, (n, parts) in self.vecs.items():
            sig += [(key, p[0].data_ptr(), p[0].dtype) for p in parts]
        return tuple(sig)

    def _build(self, dtype, device):
        code = dt_code(dtype)
        if code == L.F64:  # the float64 mode runs aerognn/f64.py on the unpacked parameters
            raise NotImplementedError("aerognn Pack: packed MFMA operands are float32 / bfloat16 / float16")
        for key, (M, K, parts) in self.mats.items():
            for p in parts:
                if p[0].dtype not in (torch.float32, torch.bfloat16, torch.float16):
                    raise TypeError(f"aerognn Pack: {key} weights are {p[0].dtype}; model and activations must "
                                    "share a float32 / bfloat16 / float16 dtype (or both be float64)")
        for key, (n, parts) in self.vecs.items():
            for p in parts:
                if p[0].dtype not in (torch.float32, torch.bfloat16, torch.float16):
                    raise TypeError(f"aerognn Pack: {key} parameters are {p[0].dtype}")
        offs = {}
        total = 0
        for key, (M, K, parts) in self.mats.items():
            nb = packed_bytes(M, K, code)
            offs[key] = (total, nb)
            total += (nb + 255) // 256 * 256
        for key, (n, parts) in self.vecs.items():
            nb = 4 * n
            offs[key] = (total, nb)
            total += (nb + 255) // 256 * 256
        self.ws = torch.zeros(max(total, 256), dtype=torch.uint8, device=device)
        base = self.ws.data_ptr()
        descs = []
        maxthr = 1
        for key, (M, K, parts) in self.mats.items():
            o, nb = offs[key]
            self.views[key] = base + o
            for (W, ro, co, tr) in parts:
                rows, cols = (W.shape[1], W.shape[0]) if tr else (W.shape[0], W.shape[1])
                d = L.PackDesc(W.data_ptr(), base + o, dt_code(W.dtype), code, rows, cols, int(tr),
                               W.stride(0), ro, co, M, K)
                descs.append(d)
                units = ((rows + 31) // 32) * ((cols + 15) // 16) * (2 if code == L.F32 else 1)
                maxthr = max(maxthr, units * 64)
        for key, (n, parts) in self.vecs.items():
            o, nb = offs[key]
            self.views[key] = base + o
            for (v, off) in parts:
                descs.append(L.PackDesc(v.data_ptr(), base + o, dt_code(v.dtype), L.F32, 0, v.numel(), 0, v.stride(0),
                                        0, int(off), 0, n))
                maxthr = max(maxthr, v.numel())
        raw = (L.PackDesc * len(descs))(*descs)
        host = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8)
        self._descs = host.to(device)
        self._ndesc = len(descs)
        self._maxthr = maxthr

    def update(self, dtype, device):
        for key, (M, K, parts) in self.mats.items():
            for p in parts:
                if p[0].dim() != 2 or p[0].stride(1) != 1:
                    raise RuntimeError("aerognn: packed weights need unit column stride (rows may be strided)")
        sig = self._signature(dtype)
        if sig != self._sig:
            self._build(dtype, device)
            self._sig = sig
        check(L.lib().agn_pack(self._descs.data_ptr(), self._ndesc, self._maxthr, stream()), "pack")
        return self

    def __getitem__(self, key):
        return self.views[key]


# ----------------------------------------------------------------------------- fused MLP chain
def mlp_forward(*, rows, dtype, hidden, nlin, out_dim, segs, wpk, bias, out, out_ld=None,
                ln=None, proj=None, src=None, dst=None, resid=None, acts=None, hpre=None, stats=None,
                tag=None, cost=None, act_fn=0):
    """segs: list of (kind, k, ld, tensor, index_tensor, store_tensor); act_fn: AGN_ACT_* (L.ACT)."""
    a = L.MlpFwdArgs()
    a.rows, a.dtype, a.hidden, a.nlin = rows, dt_code(dtype), hidden, nlin
    a.act_fn = act_fn
    a.out_dim, a.nseg = out_dim, len(segs)
    a.use_ln = 1 if ln is not None else 0
    a.out_ld = out_ld if out_ld is not None else out_dim
    for i, (kind, k, ld, t, idx, store) in enumerate(segs):
        a.seg[i] = L.Seg(kind, k, ld, 0, ptr(t), ptr(idx), ptr(store))
    for i in range(nlin):
        a.wpk[i] = wpk[i]
        a.bias[i] = bias[i]
    if ln is not None:
        a.ln_g, a.ln_b = ln
    a.proj, a.src, a.dst = ptr(proj), ptr(src), ptr(dst)
    a.resid, a.out = ptr(resid), ptr(out)
    if acts is not None:
        for i, t in enumerate(acts):
            a.act[i] = ptr(t)
            a.mask[i] = ptr(_mask_of(t))
            a.pre[i] = ptr(_pre_of(t))
    a.hpre, a.stats = ptr(hpre), ptr(stats)
    a.tiled = int(any(is_tiled(t) for t in list(acts or []) + [hpre]))
    with timed(tag, cost):
        check(L.lib().agn_mlp_forward(C.byref(a), stream()), "mlp_forward")


# The persistent projection kernels (csrc/proj.hip) for the sum-trick edge block's node-row
# GEMMs; bitwise identical to the general-kernel path, which AEROGNN_PROJ_KERNEL=0 selects.
def proj_kernel_ok(x, H):
    import os
    return (os.environ.get("AEROGNN_PROJ_KERNEL", "1") != "0" and x.dtype == torch.bfloat16 and H == 128
            and x.dim() == 2 and x.shape[1] == 128 and x.stride(1) == 1)


def proj_forward(rows, x, wpk, bias, out, tag=None, cost=None):
    with timed(tag, cost):
        check(L.lib().agn_proj_forward(rows, ptr(x), x.stride(0), wpk, bias, ptr(out), out.stride(0), stream()),
              "proj_forward")


def proj_backward(rows, dps, dpd, wtpk, dx, tag=None, cost=None):
    assert dps.stride(0) == dpd.stride(0)
    with timed(tag, cost):
        check(L.lib().agn_proj_backward(rows, ptr(dps), ptr(dpd), dps.stride(0), wtpk, ptr(dx), dx.stride(0),
                                        stream()), "proj_backward")


def bwd_nblocks(rows):
    return int(L.lib().agn_mlp_bwd_nwaves(int(rows)))


def mlp_backward(*, rows, dtype, hidden, nlin, out_dim, in_dim, wtpk, acts, g, gpre,
                 ln_g=None, hpre=None, stats=None, g2=None, gidx=None, din=(), ln_partial=None,
                 tag=None, cost=None, act_fn=0):
    """din: list of (k, tensor_or_None, resid_flag); act_fn: the forward's AGN_ACT_*."""
    a = L.MlpBwdArgs()
    a.rows, a.dtype, a.hidden, a.nlin = rows, dt_code(dtype), hidden, nlin
    a.act_fn = act_fn
    a.out_dim, a.in_dim = out_dim, in_dim
    a.use_ln = 1 if ln_g is not None else 0
    for i in range(nlin):
        a.wtpk[i] = wtpk[i]
        a.gpre[i] = ptr(gpre[i]) if gpre[i] is not None else None
    for i, t in enumerate(acts):
        a.act[i] = ptr(t)
        a.mask[i] = ptr(_mask_of(t))
        a.pre[i] = ptr(_pre_of(t))
    a.hpre, a.stats, a.ln_g = ptr(hpre), ptr(stats), ln_g
    a.g, a.g2, a.gidx = ptr(g), ptr(g2), ptr(gidx)
    a.tiled = int(any(is_tiled(t) for t in list(acts or []) + [hpre]))
    a.gpre_tiled = sum(1 << l for l in range(nlin) if is_tiled(gpre[l]))
    a.din_nseg = len(din)
    for i, (k, t, r) in enumerate(din):
        a.din_k[i] = k
        a.din[i] = ptr(t)
        a.din_resid[i] = int(r)
    a.ln_partial = ptr(ln_partial)
    with timed(tag, cost):
        check(L.lib().agn_mlp_backward(C.byref(a), stream()), "mlp_backward")
    return a.ln_rows


# AEROGNN_CHECK_FAULTS=1 (set by the test suite): read the device fault word after every
# persistent hand-off launch (a device synchronisation each time; never on the timed path).
CHECK_FAULTS = __import__("os").environ.get("AEROGNN_CHECK_FAULTS", "0") == "1"
STAMPS = None  # diagnostics: a uint64 device tensor of 2*8*8*16 entries (a -DAGN_EB_STAMPS library)


def fused_edge_train_ok(rows, dtype, hidden, nlin, has_ln):
    """agn_edge_bwd_fused applies: bf16 H=128 sum-trick edge chains (W_e + 3 Linears + LN) large
    enough for the persistent kernels. Then the training forward saves only a1 and the LayerNorm
    statistics of the edge chain (edge_saves_ok) and one launch recomputes the rest in the backward
    (csrc/edge_bwd.hip): 414 instead of 680 GB of HBM traffic per C3 train step (DESIGN.md §9,
    rounds 3 and 6). AEROGNN_FUSED_EDGE_BWD=0 selects the split path (saved activations,
    agn_mlp_backward + agn_wgrad) for A/B tests."""
    import os
    return (os.environ.get("AEROGNN_FUSED_EDGE_BWD", "1") != "0" and dtype == torch.bfloat16 and hidden == 128
            and nlin == 4 and has_ln and rows >= 64 * 1024)


def edge32_ok(dtype, hidden, nlin, has_ln, act=0):
    """agn_edge_forward32 (csrc/edge32_fwd.hip) applies to the bf16 H=128 sum-trick ReLU edge chain
    (W_e + 3 Linears + LN); AEROGNN_EDGE32=0 turns it off (then the resident agn_mlp_forward kernel
    runs, bitwise the same outputs)."""
    import os
    return (os.environ.get("AEROGNN_EDGE32", "1") != "0" and dtype == torch.bfloat16 and hidden == 128
            and nlin == 4 and has_ln and act == 0)


def edge_saves_ok():
    """The training forward saves a1 and the LayerNorm statistics for the fused backward
    (agn_edge_forward32 act[0] / stats), which then starts its recompute at Lin1 (DESIGN.md §9,
    round 6). AEROGNN_EB_SAVED=0: save nothing, recompute h0 from e and the projection rows."""
    import os
    return os.environ.get("AEROGNN_EB_SAVED", "1") != "0"


def edge_forward(*, rows, wpk, bias, ln, e, proj, src, dst, out, a1=None, stats=None, tag=None, cost=None):
    """agn_edge_forward32: out = e + LN(chain(e, P_s[src] + P_d[dst])) on 32-row tiles (bitwise the
    resident agn_mlp_forward kernel); a1 (AGN_TILED, tiled_empty) and stats ([rows, 2] fp32) are the
    fused backward's training saves, both or neither."""
    lib = L.lib()
    a = L.EdgeFwdArgs()
    a.rows = int(rows)
    a.nblk = int(lib.agn_edge_fwd32_blocks(int(rows)))
    for i in range(4):
        a.wpk[i] = wpk[i]
        a.bias[i] = bias[i]
    a.ln_g, a.ln_b = ln
    a.e, a.proj, a.src, a.dst, a.out = ptr(e), ptr(proj), ptr(src), ptr(dst), ptr(out)
    a.act[0] = ptr(a1)
    a.stats = ptr(stats)
    with timed(tag, cost):
        check(lib.agn_edge_forward32(C.byref(a), stream()), "edge_forward32")


# Production-path fault polling: every FAULT_POLL_EVERY fused launches an async copy
# of the device fault word goes to page-locked host memory (agn_fault_status_async, no device
# synchronisation); a later launch reads it once the copy's event has completed. At every optimizer
# step (a global step pre-hook, registered with the first fused launch) fault_checkpoint() raises on a
# completed copy and enqueues one that covers the launches since the last, so the final <= 15 launches
# of a run are read too; an atexit hook waits for the last copy. A copy read
# inside a backward only records the word: the raise happens at the step boundary (optimizer step,
# GradAllReduce.__call__, exit). A fault is fatal to the job: under torchrun the raising rank's exit
# ends the other ranks (they would otherwise wait in the next all-reduce).
FAULT_POLL_EVERY = 16
_fault = {"buf": None, "event": None, "n": 0, "dirty": False, "hooked": False, "word": 0}


def _fault_read(block, defer=False):
    """Read a completed copy of the fault word. defer=True (inside a backward) only records a
    nonzero word; the next step boundary raises it, so no rank stops in the middle of its backward
    with all-reduce buckets in flight."""
    st = _fault
    ev = st["event"]
    if ev is not None and (block or ev.query()):
        if block:
            ev.synchronize()
        st["word"] |= int(st["buf"][0])
        st["event"] = None
    f = st["word"]
    if f and not defer:
        raise L.AeroGNNError(f"fused edge backward: device fault word {f:#x} (LDS ring wait timed out; "
                             "dW of a recent step invalid)")


def _fault_enqueue():
    st = _fault
    if st["buf"] is None:
        st["buf"] = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    check(L.lib().agn_fault_status_async(C.c_void_p(st["buf"].data_ptr()), stream()), "fault_status_async")
    ev = torch.cuda.Event()
    ev.record()
    st["event"] = ev
    st["n"] = 0
    st["dirty"] = False


def fault_checkpoint(block=False):
    """Step boundary: raise if a completed copy of the fault word is nonzero, then enqueue a copy
    covering every fused launch so far (if any ran since the last); block=True waits for it and
    raises on a fault (the end of a run)."""
    _fault_read(False)
    if _fault["dirty"]:
        if _fault["event"] is not None:  # the previous copy first (one buffer)
            _fault_read(True)
        _fault_enqueue()
    if block:
        _fault_read(True)


def _step_pre_hook(_opt, _args, _kwargs):
    fault_checkpoint()


def _exit_check():
    try:
        fault_checkpoint(block=True)
    except L.AeroGNNError as exc:
        import sys
        print(f"aerognn: {exc}", file=sys.stderr)
        raise


def _poll_faults():
    st = _fault
    if not st["hooked"]:
        import atexit
        from torch.optim.optimizer import register_optimizer_step_pre_hook
        register_optimizer_step_pre_hook(_step_pre_hook)
        atexit.register(_exit_check)
        st["hooked"] = True
    _fault_read(False, defer=True)
    st["dirty"] = True
    st["n"] += 1
    if st["event"] is None and st["n"] >= FAULT_POLL_EVERY:
        _fault_enqueue()


def edge_bwd_fused(*, rows, wpk, wtpk0, bias, ln_g, e, proj, src, dst, g, g2, de, g0, tag=None, cost=None,
                   a1=None, stats=None, scratch=None):
    """agn_edge_bwd_fused; returns (dW1..dW3 [3,128,128] fp32, db1..db3 [3,128] fp32, LayerNorm
    partials [nblk, 256] fp32, nblk) after the fixed-order slab reduction (agn_wgrad_reduce).
    a1 / stats: the forward's saves (agn_edge_forward32);
    then e, proj and src are not read. scratch None: AEROGNN_EB_SCRATCH (default off) decides whether
    a2 goes through a scratch buffer instead of a second recompute on the recompute path (with a1 /
    stats, a2 and a3 stay in registers; bitwise the same outputs; not faster, and its slices leave L2:
    DESIGN.md §9 round 6)."""
    import os
    lib = L.lib()
    dev = g2.device
    H = 128
    nblk = int(lib.agn_edge_bwd_blocks(int(rows)))
    dwp = torch.empty(3 * nblk * H * H, dtype=torch.float32, device=dev)
    dbp = torch.empty(3 * nblk * H, dtype=torch.float32, device=dev)
    lnp = torch.empty(nblk, 2 * H, dtype=torch.float32, device=dev)
    if scratch is None:
        scratch = os.environ.get("AEROGNN_EB_SCRATCH", "0") == "1"
    scr = (torch.empty(int(lib.agn_edge_bwd_scratch_bytes(nblk)), dtype=torch.uint8, device=dev)
           if scratch else None)
    a = L.EdgeBwdArgs()
    a.rows, a.nblk = int(rows), nblk
    for i in range(4):
        a.wpk[i] = wpk[i]
        a.bias[i] = bias[i]
    a.ln_g = ln_g
    a.e, a.proj, a.src, a.dst = ptr(e), ptr(proj), ptr(src), ptr(dst)
    a.g, a.g2 = ptr(g), ptr(g2)
    a.de, a.g0, a.dw_partial, a.db_partial, a.ln_partial = ptr(de), ptr(g0), ptr(dwp), ptr(dbp), ptr(lnp)
    a.stamps = ptr(STAMPS)
    a.a1, a.stats, a.scratch = ptr(a1), ptr(stats), ptr(scr)
    a.wtpk0 = wtpk0  # W_e^T packed (ChainSpec.wtpk()[0])
    with timed(tag, cost):
        check(lib.agn_edge_bwd_fused(C.byref(a), stream()), "edge_bwd_fused")
    if CHECK_FAULTS:  # tests / debug runs: a bounded ring wait that gave up is an error, not wrong dW
        f = L.fault_status(reset=True)
        if f:
            raise L.AeroGNNError(f"agn_edge_bwd_fused: device fault word {f:#x} (LDS ring wait timed out; dW invalid)")
    else:
        _poll_faults()
    return _reduce_slabs(rows, dwp, dbp, lnp, nblk, dev)


def _reduce_slabs(rows, dwp, dbp, lnp, nblk, dev):
    """dW1..dW3 / db1..db3 from a fused backward's per-block slabs (fixed order, agn_wgrad_reduce)."""
    H = 128
    dw = torch.empty(3, H, H, dtype=torch.float32, device=dev)
    db = torch.empty(3, H, dtype=torch.float32, device=dev)
    b = L.WgradBatch()
    b.n = 3
    for l in range(3):
        b.d[l] = L.WgradDesc(None, None, H, H, H, H, int(rows), H, ptr(dwp[l * nblk * H * H:]), ptr(dbp[l * nblk * H:]),
                             ptr(dw[l]), ptr(db[l]), 0, 0, nblk, 0)
    check(L.lib().agn_wgrad_reduce(C.byref(b), nblk, stream()), "wgrad_reduce")
    return dw, db, lnp, nblk


def encoder_fused_ok(spec, dtype, k, rows, need_dx):
    """agn_encoder_bwd_fused applies (training): a bf16 encoder MLP of 4 Linears (k <= 16 inputs, H = 128
    hidden and out, ReLU, LayerNorm) on >= 65,536 rows whose input needs no gradient (the model's
    node / edge features). Then the forward saves nothing and the backward recomputes the chain on
    chip with dW1..dW3 there. AEROGNN_FUSED_ENC_BWD=0 selects the split path."""
    import os
    return (os.environ.get("AEROGNN_FUSED_ENC_BWD", "1") != "0" and dtype == torch.bfloat16 and not need_dx
            and spec.hidden == 128 and spec.out_dim == 128 and spec.nlin == 4 and spec.ln is not None
            and spec.act == L.ACT["relu"] and 1 <= k <= 16 and rows >= 64 * 1024)


def encoder_bwd_fused(*, rows, wpk, bias, ln_g, x, xidx, g, g0, tag=None, cost=None):
    """agn_encoder_bwd_fused: (dW1..dW3, db1..db3, LayerNorm partials, nblk) of an encoder chain, and
    G0 into g0 ([rows, 128] row-major) for dW0 / db0; x [n, k] bf16 (rows gathered by xidx, int32,
    when given)."""
    lib = L.lib()
    dev = g.device
    H = 128
    nblk = int(lib.agn_edge_bwd_blocks(int(rows)))
    dwp = torch.empty(3 * nblk * H * H, dtype=torch.float32, device=dev)
    dbp = torch.empty(3 * nblk * H, dtype=torch.float32, device=dev)
    lnp = torch.empty(nblk, 2 * H, dtype=torch.float32, device=dev)
    import os
    scr = (torch.empty(int(lib.agn_edge_bwd_scratch_bytes(nblk)), dtype=torch.uint8, device=dev)
           if os.environ.get("AEROGNN_EB_SCRATCH", "0") == "1" else None)
    a = L.EdgeBwdArgs()
    a.rows, a.nblk = int(rows), nblk
    for i in range(4):
        a.wpk[i] = wpk[i]
        a.bias[i] = bias[i]
    a.ln_g = ln_g
    a.e, a.src, a.g, a.g0 = ptr(x), ptr(xidx), ptr(g), ptr(g0)
    a.dw_partial, a.db_partial, a.ln_partial, a.scratch = ptr(dwp), ptr(dbp), ptr(lnp), ptr(scr)
    a.xk, a.xld = int(x.shape[1]), int(x.stride(0))
    a.stamps = ptr(STAMPS)
    with timed(tag, cost):
        check(lib.agn_encoder_bwd_fused(C.byref(a), stream()), "encoder_bwd_fused")
    if CHECK_FAULTS:
        f = L.fault_status(reset=True)
        if f:
            raise L.AeroGNNError(f"agn_encoder_bwd_fused: device fault word {f:#x} (LDS ring wait timed out; dW invalid)")
    else:
        _poll_faults()
    return _reduce_slabs(rows, dwp, dbp, lnp, nblk, dev)


def reduce_partials(partial, nw, n, out):
    check(L.lib().agn_reduce_partials(ptr(partial), nw, n, ptr(out), stream()), "reduce_partials")


def segment_sum(rows, k, ptr_t, perm, src, out, mean=False, src_ld=None, out_ld=None):
    check(L.lib().agn_segment_sum(rows, k, dt_code(src.dtype), ptr(ptr_t), ptr(perm), ptr(src),
                                  src_ld or src.stride(0), ptr(out), out_ld or out.stride(0), int(mean),
                                  stream()), "segment_sum")
    return out


def segment_sum2(rows, k, base, a, b, out):
    """out = base + segment sums of a = (ptr, perm, src) + of b, fp32 in that order (out may be
    base; base None = 0)."""
    (pa, qa, sa), (pb, qb, sb) = a, b
    check(L.lib().agn_segment_sum2(rows, k, dt_code(sa.dtype), ptr(base), base.stride(0) if base is not None else 0, ptr(pa), ptr(qa), ptr(sa),
                                   sa.stride(0), ptr(pb), ptr(qb), ptr(sb), sb.stride(0), ptr(out), out.stride(0),
                                   stream()), "segment_sum2")
    return out


def segment_max(rows, k, ptr_t, perm, src, out, argmax):
    check(L.lib().agn_segment_max(rows, k, dt_code(src.dtype), ptr(ptr_t), ptr(perm), ptr(src), src.stride(0), ptr(out),
                                  out.stride(0), ptr(argmax), stream()), "segment_max")
    return out


def segment_max_backward(rows, k, argmax, gout, dx):
    check(L.lib().agn_segment_max_backward(rows, k, dt_code(gout.dtype), ptr(argmax), ptr(gout), gout.stride(0), ptr(dx),
                                           dx.stride(0), stream()), "segment_max_backward")
    return dx


def gather_rows(rows, k, idx, src, out, cnt_ptr=None, add=None):
    check(L.lib().agn_gather_rows(rows, k, dt_code(src.dtype), ptr(idx), ptr(src), src.stride(0),
                                  ptr(cnt_ptr), ptr(add), add.stride(0) if add is not None else 0,
                                  ptr(out), out.stride(0), stream()), "gather_rows")
    return out


def scatter_rows(idx32, src, out):
    """out[idx[r]] = src[r] (rows of `src` in order; idx unique)."""
    check(L.lib().agn_scatter_rows(idx32.numel(), src.shape[1], dt_code(src.dtype), ptr(idx32), ptr(src),
                                   src.stride(0), ptr(out), out.stride(0), stream()), "scatter_rows")
    return out


def colsum_rows(p, nw, n, out):
    """out[c] = sum_r p[r][c] over nw rows, deterministic 2-level reduction (LN parameter grads)."""
    sr = min(512, max(1, nw))
    scratch = torch.empty(sr * n, dtype=torch.float32, device=p.device)
    check(L.lib().agn_colsum(ptr(p), nw, n, ptr(scratch), sr, ptr(out), stream()), "colsum")
    return out


class WGrad:
    """Batched weight/bias gradients dW = G^T X (fp32), db = colsum(G) on libaerognn.

    add(G, X, dw_view, db) queues one Linear (dw_view: fp32 [M][>=K] view, may be a column
    slice of a wider dW); run() launches ceil(n/8) kernels (+ their fixed-order reductions).
    """

    def __init__(self, tag="wgrad"):
        self.items = []
        # kernel-table tag of the launches (bench.py): wgrad_edge (E-row edge chains), wgrad_node
        # (W_s / W_d and the node MLP), wgrad_enc (encoders, decoder, other MLPs)
        self.tag = tag

    def add(self, G, X, dw, db=None, xidx=None):
        """xidx: X is gathered, row r of the operand = X[xidx[r]] (int32, one entry per row of G)."""
        assert G.dtype == X.dtype and logical_rows(G) == (logical_rows(X) if xidx is None else xidx.numel())
        assert dw.dtype == torch.float32 and dw.stride(1) == 1
        assert xidx is None or (xidx.dtype == torch.int32 and not is_tiled(X))
        self.items.append((G, X, dw, db, xidx))

    def run(self):
        lib = L.lib()
        # gathered-operand descs launch on their own: one xidx desc puts the whole launch on the
        # gathered instantiation, and mixing them measured slower than two launches (2.07 against
        # 0.67 + 1.07 ms for the C3 edge encoder)
        plain = [it for it in self.items if it[4] is None]
        gath = [it for it in self.items if it[4] is not None]
        chunks = [grp[i:i + L.MAX_WGRAD] for grp in (plain, gath) for i in range(0, len(grp), L.MAX_WGRAD)]
        for chunk in chunks:
            dev = chunk[0][0].device
            live = []
            for G, X, dw, db, xi in chunk:
                if logical_rows(G) == 0:
                    dw.zero_()
                    if db is not None:
                        db.zero_()
                else:
                    live.append((G, X, dw, db, xi))
            if not live:
                continue
            b = L.WgradBatch()
            b.n = len(live)
            for j, (G, X, dw, db, xi) in enumerate(live):
                b.d[j] = L.WgradDesc(ptr(G), ptr(X), G.stride(0), X.stride(0), G.shape[1], X.shape[1], logical_rows(G),
                                     dw.stride(0), None, None, ptr(dw), ptr(db), int(is_tiled(G)), int(is_tiled(X)), 0, 0,
                                     ptr(xi))
            check(lib.agn_wgrad_plan(C.byref(b)), "wgrad_plan")  # one uniform split count, from the largest desc
            sizes = [int(lib.agn_wgrad_partial_floats(G.shape[1], X.shape[1], b.d[j].nsplit))
                     for j, (G, X, _, _, _) in enumerate(live)]
            bsz = [b.d[j].nsplit * ((G.shape[1] + 127) // 128) * 128 if db is not None else 0
                   for j, (G, _, _, db, _) in enumerate(live)]
            scratch = torch.empty(sum(sizes) + sum(bsz), dtype=torch.float32, device=dev)
            o = 0
            for j, (G, X, dw, db, _) in enumerate(live):
                b.d[j].dw_partial = ptr(scratch[o:o + sizes[j]])
                o += sizes[j]
                if db is not None:
                    b.d[j].db_partial = ptr(scratch[o:o + bsz[j]])
                    o += bsz[j]
            # operator I/O: G and X read once per row (+ the fp32 dW / db written); its SURVEY §8(d)
            # share is 0 (a fused backward keeps G in registers), so the alg_bytes slot carries 0
            s_el = live[0][0].element_size()
            io = sum(logical_rows(G) * (G.shape[1] + X.shape[1]) * s_el + 4 * G.shape[1] * (X.shape[1] + 1)
                     for G, X, _, _, _ in live)
            fl = sum(2.0 * logical_rows(G) * G.shape[1] * X.shape[1] for G, X, _, _, _ in live)
            with timed(self.tag, (0.0, fl, io)):
                check(lib.agn_wgrad(C.byref(b), dt_code(live[0][0].dtype), 0, stream()), "wgrad")
        self.items = []


# --------------------------------------------------------------------------- algorithmic costs
# Each tagged launch records (alg_bytes, flops, impl_bytes):
#   alg_bytes  = the launch's share of SURVEY §8(d)'s fully-fused per-layer minimum
#                B = E(2sH + 8) + N(8sH): edge kernel E(2sH + 8) + N(2sH) (P_s/P_d rows read once),
#                projection N(3sH) (read x, write P_s|P_d), node kernel N(3sH) (read x, agg, write x');
#                training = 3x forward, so each backward kernel carries 2x its forward share;
#   impl_bytes = the bytes this implementation's kernel must move (its own I/O model, cost_* below).
def alg8d_edge(E, N, H, s, bwd=False):
    return (2 if bwd else 1) * (E * (2 * s * H + 8) + N * 2 * s * H)


def alg8d_node(N, H, s, bwd=False, proj=False):
    return (2 if bwd else 1) * N * 3 * s * H * (2 if (bwd and proj) else 1)


def with_alg(alg, impl):
    """(alg_bytes, flops, impl_bytes) from a §8(d) share and an implementation cost tuple."""
    return (alg, impl[1], impl[0])


def mask_bytes(H):
    """AGN_RELU_MASK bytes per row of one hidden layer (8 B per lane pair and dword)."""
    return 8 * max(1, (H + 63) // 64)


def cost_edge_fwd(E, N, H, s, nlin, train, a1_saves=False):
    """Minimum HBM bytes / MFMA flops of one fused edge-MLP launch;
    a1_saves: agn_edge_forward32's training saves for the fused backward (a1 + statistics)."""
    per = 2 * H * s + 8 + ((nlin - 1) * (H * s + mask_bytes(H)) + H * s + 8 if train else 0)
    per += (H * s + 8) if a1_saves else 0
    return E * per + N * 2 * H * s, 2 * E * H * H * nlin


def cost_node_fwd(E, N, H, s, nlin, train):
    per = 2 * H * s + 8 + ((nlin - 1) * (H * s + mask_bytes(H)) + 2 * H * s + 8 if train else 0)
    return N * per + E * H * s, 2 * N * H * (2 * H + (nlin - 1) * H)


def cost_proj(N, H, s):
    return N * 3 * H * s, 2 * N * H * 2 * H


def cost_edge_bwd(E, N, H, s, nlin):
    # g, g2[dst], masks, hpre, stats, gpre writes, de, dst index
    per = H * s + H * s + (nlin - 1) * mask_bytes(H) + H * s + 8 + nlin * H * s + H * s + 4
    return E * per + N * H * s, 2 * E * H * H * nlin


def cost_edge_fwd_cat(E, N, H, s, nlin, train):
    """Concat edge MLP (EdgeBlock / GMP): e and the two gathered node rows in, e' (+ saves) out."""
    per = 4 * H * s + 8 + ((nlin - 1) * (H * s + mask_bytes(H)) + H * s + 8 if train else 0)
    return E * per, 2 * E * H * (3 * H + (nlin - 1) * H)


def cost_edge_bwd_cat(E, N, H, s, nlin):
    per = H * s + H * s + (nlin - 1) * mask_bytes(H) + H * s + 8 + nlin * H * s + 3 * H * s + 4
    return E * per + N * H * s, 2 * E * H * (3 * H + (nlin - 1) * H)


def cost_wec_fwd(E, N, out, s, hid=64):
    """WeightedEdgeConv forward: per edge src/perm ids, P_a[src] and Tx[src] gathers, both
    positions, the weight write; per receiver P_b, rowptr and the output row."""
    return E * (12 + hid * s + out * s + 24 + s) + N * (8 + hid * s + out * s), E * (2 * hid + 2 * out + 16)


def cost_wec_bwd(E, N, out, s, hid=64):
    dst = E * (12 + out * s + hid * s + 24 + 4 + 4 * hid) + N * (out * s + 2 * hid * s)
    src = E * (12 + out * s + 4 * hid) + N * (8 + out * s + hid * s)
    return dst + src, E * (4 * hid + 4 * out)


def cost_node_bwd(N, H, s, nlin):
    per = H * s + H * s + (nlin - 1) * mask_bytes(H) + 8 + nlin * H * s + 2 * H * s  # g, hpre, masks, ...
    return N * per, 2 * N * H * (H * (nlin - 1) + 2 * H)


def cost_edge_bwd_fused(E, N, H, s, saved=False):
    """agn_edge_bwd_fused: per edge the ids, e, the sender's projection row, g, and de + G0 written
    (+ the row re-reads of g for de, L2); per receiver its P_d row and dAgg row. saved: a1 and the
    statistics instead of e and the projection rows (one Linear fewer recomputed)."""
    if saved:
        per = 4 + 8 + H * s * 2 + H * s * 2
        return E * per + N * H * s, 2 * E * H * H * (3 + 4 + 3)
    per = 8 + H * s * 3 + H * s * 2
    flops = 2 * E * H * H * (4 + 2 + 4 + 3)  # forward 4 + recompute 2 + dX 4 + dW 3 Linears
    return E * per + N * 2 * H * s, flops
