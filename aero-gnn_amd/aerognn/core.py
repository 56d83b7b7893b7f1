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


def dt_code(dtype) -> int:
    if dtype == torch.float32:
        return L.F32
    if dtype == torch.bfloat16:
        return L.BF16
    raise NotImplementedError(f"aerognn kernels compute in float32 or bfloat16, got {dtype}")


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
                descs.append(L.PackDesc(v.data_ptr(), base + o, dt_code(v.dtype), L.F32, 0, v.numel(), 0, 1,
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
                if not p[0].is_contiguous():
                    raise RuntimeError("aerognn: packed weights must be contiguous")
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
                ln=None, proj=None, src=None, dst=None, resid=None, acts=None, hpre=None, stats=None):
    """segs: list of (kind, k, ld, tensor, index_tensor, store_tensor)."""
    a = L.MlpFwdArgs()
    a.rows, a.dtype, a.hidden, a.nlin = rows, dt_code(dtype), hidden, nlin
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
    a.hpre, a.stats = ptr(hpre), ptr(stats)
    check(L.lib().agn_mlp_forward(C.byref(a), stream()), "mlp_forward")


def bwd_nblocks(rows):
    return int(L.lib().agn_mlp_bwd_nwaves(int(rows)))


def mlp_backward(*, rows, dtype, hidden, nlin, out_dim, in_dim, wtpk, acts, g, gpre,
                 ln_g=None, hpre=None, stats=None, g2=None, gidx=None, din=(), ln_partial=None):
    """din: list of (k, tensor_or_None, resid_flag)."""
    a = L.MlpBwdArgs()
    a.rows, a.dtype, a.hidden, a.nlin = rows, dt_code(dtype), hidden, nlin
    a.out_dim, a.in_dim = out_dim, in_dim
    a.use_ln = 1 if ln_g is not None else 0
    for i in range(nlin):
        a.wtpk[i] = wtpk[i]
        a.gpre[i] = ptr(gpre[i]) if gpre[i] is not None else None
    for i, t in enumerate(acts):
        a.act[i] = ptr(t)
    a.hpre, a.stats, a.ln_g = ptr(hpre), ptr(stats), ln_g
    a.g, a.g2, a.gidx = ptr(g), ptr(g2), ptr(gidx)
    a.din_nseg = len(din)
    for i, (k, t, r) in enumerate(din):
        a.din_k[i] = k
        a.din[i] = ptr(t)
        a.din_resid[i] = int(r)
    a.ln_partial = ptr(ln_partial)
    check(L.lib().agn_mlp_backward(C.byref(a), stream()), "mlp_backward")


def reduce_partials(partial, nw, n, out):
    check(L.lib().agn_reduce_partials(ptr(partial), nw, n, ptr(out), stream()), "reduce_partials")


def segment_sum(rows, k, ptr_t, perm, src, out, mean=False, src_ld=None, out_ld=None):
    check(L.lib().agn_segment_sum(rows, k, dt_code(src.dtype), ptr(ptr_t), ptr(perm), ptr(src),
                                  src_ld or src.stride(0), ptr(out), out_ld or out.stride(0), int(mean),
                                  stream()), "segment_sum")
    return out


def gather_rows(rows, k, idx, src, out, cnt_ptr=None, add=None):
    check(L.lib().agn_gather_rows(rows, k, dt_code(src.dtype), ptr(idx), ptr(src), src.stride(0),
                                  ptr(cnt_ptr), ptr(add), add.stride(0) if add is not None else 0,
                                  ptr(out), out.stride(0), stream()), "gather_rows")
    return out


def wgrad(G, X, out=None):
    """dW = G^T X accumulated in fp32 (G: [rows, M], X: [rows, K])."""
    if G.shape[0] == 0:
        return torch.zeros(G.shape[1], X.shape[1], dtype=torch.float32, device=G.device)
    if G.dtype == torch.float32:
        return torch.mm(G.t(), X, out=out) if out is not None else torch.mm(G.t(), X)
    return torch.mm(G.t(), X, out_dtype=torch.float32)


def colsum(G):
    return G.sum(0, dtype=torch.float32)
