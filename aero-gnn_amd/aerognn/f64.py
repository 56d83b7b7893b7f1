"""float64 mode (train.py:20-40, precision "double" / "float64") of the MLP / GMP path.

torch.set_default_dtype(torch.float64) makes every parameter and activation fp64. The bf16 / fp32
kernels' MFMA tiles have no fp64 counterpart on CDNA4, so this mode runs on the agn_f64_* kernels
(csrc/f64.hip: LDS-tiled FMA GEMM with gather / addend / ReLU / ReLU-mask epilogues, split-row
dW with a fixed-order reduction, LayerNorm) plus the graph ops' float64 instantiations
(agn_segment_sum / agn_gather_rows / agn_scatter_rows with AGN_F64). Nothing here computes on
the CPU or through torch operators; the autograd Functions below call the library only.

    MLP64Fn   one Linear / ReLU / ... / LayerNorm chain (models/mlp.py:40-51, the EdgeBlockSum
              chain of mgnLayer.py:72-105), inputs as column segments (optionally row-gathered:
              x[src], x[dst] of the concat EdgeBlock, mgnLayer.py:30-49) and gathered addends
              (the sum trick's (W_s x)[src] and (W_d x + b)[dst]), an optional residual
              (mgnLayer.py:205, 209) added after the LayerNorm
    SegSum64Fn  scatter_add / scatter_mean over a level's receivers (mgnLayer.py:144-148)
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from ._lib import check, ptr
from .core import require_device, segment_sum, gather_rows, stream

F64 = torch.float64


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def gemm(rows, n, segs, out, bias=None, adds=(), mask=None, relu=False, act=None, mask_act=0, pre_out=None):
    """out[rows][n] = f?(mask?(sum over segs of A . B + bias + adds)). segs: (a, aidx, k, w,
    transw) with B(j, c) = w[c][j] (transw) or w[j][c]; adds: (t, idx) addends [*, n].
    f: relu=True, or act = an AGN_ACT_* code (its pre-activation also to pre_out when given);
    mask_act: 0 = ReLU backward on the saved activation `mask`, 1 + AGN_ACT_* = out *= f'(mask)
    with `mask` the saved pre-activation."""
    if rows == 0:
        return out
    a = L.F64GemmArgs()
    a.rows, a.n, a.nseg = int(rows), int(n), len(segs)
    for i, (x, idx, k, w, transw) in enumerate(segs):
        a.seg[i] = L.F64Seg(ptr(x), ptr(idx), x.stride(0), int(k), ptr(w), w.stride(0), int(transw))
    a.bias = ptr(bias)
    for q, (t, idx) in enumerate(adds):
        a.add[q], a.add_idx[q], a.add_ld[q] = ptr(t), ptr(idx), t.stride(0)
    a.mask = ptr(mask)
    a.mask_ld = mask.stride(0) if mask is not None else 0
    a.mask_act = int(mask_act)
    a.relu = 1 + int(act) if act is not None else int(relu)
    a.pre_out, a.pre_ld = ptr(pre_out), pre_out.stride(0) if pre_out is not None else 0
    a.out, a.out_ld = ptr(out), out.stride(0)
    check(L.lib().agn_f64_gemm(C.byref(a), stream()), "f64_gemm")
    return out


def wgrad(g, x, xidx, dw, db=None):
    """dw[m][k] = g^T x[xidx] (dw may be a column slice of a wider dW), db = colsum g."""
    a = L.F64WgradArgs()
    a.rows, a.m, a.k = g.shape[0], g.shape[1], dw.shape[1]
    a.g, a.ldg = ptr(g), g.stride(0)
    a.x, a.ldx, a.xidx = ptr(x), x.stride(0), ptr(xidx)
    a.dw, a.ldw, a.db = ptr(dw), dw.stride(0), ptr(db)
    lib = L.lib()
    nb = int(lib.agn_f64_wgrad_scratch_bytes(C.byref(a)))
    scratch = torch.empty(max(nb // 8, 1), dtype=F64, device=g.device)
    check(lib.agn_f64_wgrad(C.byref(a), ptr(scratch), stream()), "f64_wgrad")


def scatter_rows_sum(d, idx, nrows):
    """out[r] = sum over i with idx[i] == r of d[i] (fixed order: the grouped index's)."""
    from .graph import group_by
    perm, rp = group_by(idx, nrows)
    out = torch.empty(nrows, d.shape[1], dtype=F64, device=d.device)
    return segment_sum(nrows, d.shape[1], rp, perm, d, out)


class Chain:
    """A Linear / activation chain + optional LayerNorm bound to fp64 parameters: lins = [(W, b), ...],
    act = the AGN_ACT_* code between the Linears (mlp.py:37)."""

    def __init__(self, lins, ln=None, eps=1e-5, act=0):
        self.lins, self.ln, self.eps, self.act = lins, ln, eps, act

    def params(self):
        out = []
        for w, b in self.lins:
            out.append(w)
            if b is not None:
                out.append(b)
        if self.ln is not None:
            out += list(self.ln)
        return out


class MLP64Fn(torch.autograd.Function):
    """y = LN(chain(sum_s x_s[idx_s] W0[:, cols_s]^T + adds)) + resid (see the module docstring).
    meta = (chain, idxs per segment, add idxs, rows, has_resid)."""

    @staticmethod
    def forward(ctx, meta, *ts):
        chain, idxs, add_idx, rows, has_resid = meta
        ns, na = len(idxs), len(add_idx)
        xs, adds = ts[:ns], ts[ns:ns + na]
        resid = ts[ns + na] if has_resid else None
        require_device(*xs)
        xs = [_c(x) for x in xs]
        dev = xs[0].device
        nl = len(chain.lins)
        relu = chain.act == L.ACT["relu"]
        acts, pres, z = [], [], None
        for l, (w, b) in enumerate(chain.lins):
            n = w.shape[0]
            o = torch.empty(rows, n, dtype=F64, device=dev)
            hid = l < nl - 1
            # hidden layers: the activation in the epilogue; a non-ReLU one also keeps its input
            kw = {} if not hid else ({"relu": True} if relu else
                                     {"act": chain.act, "pre_out": torch.empty(rows, n, dtype=F64, device=dev)})
            if l == 0:
                segs, k0 = [], 0
                for x, idx in zip(xs, idxs):
                    k = x.shape[1]
                    segs.append((x, idx, k, w[:, k0:k0 + k], 1))
                    k0 += k
                gemm(rows, n, segs, o, bias=b, adds=[(_c(t), i) for t, i in zip(adds, add_idx)], **kw)
            else:
                gemm(rows, n, [(acts[-1], None, acts[-1].shape[1], w, 1)], o, bias=b, **kw)
            if hid:
                acts.append(o)
                if not relu:
                    pres.append(kw["pre_out"])
            else:
                z = o
        mean = rstd = None
        if chain.ln is not None:
            g, bt = chain.ln
            n = z.shape[1]
            y = torch.empty_like(z)
            mean = torch.empty(rows, dtype=F64, device=dev)
            rstd = torch.empty(rows, dtype=F64, device=dev)
            if rows:
                r = _c(resid) if resid is not None else None
                check(L.lib().agn_f64_layernorm_fwd(rows, n, ptr(z), z.stride(0), ptr(g), ptr(bt), ptr(r),
                                                    r.stride(0) if r is not None else 0, ptr(y), y.stride(0),
                                                    ptr(mean), ptr(rstd), chain.eps, stream()), "f64_layernorm")
        else:
            if resid is not None:
                raise NotImplementedError("aerognn float64 chain: a residual needs the LayerNorm epilogue")
            y = z
        ctx.meta = meta
        ctx.nsrc = [x.shape[0] for x in xs]
        ctx.nadd = [t.shape[0] for t in adds]
        ctx.save_for_backward(*xs, *acts, z, *([mean, rstd] if chain.ln is not None else []), *pres)
        return y

    @staticmethod
    def backward(ctx, gy):
        chain, idxs, add_idx, rows, has_resid = ctx.meta
        ns, na, nl = len(idxs), len(add_idx), len(chain.lins)
        saved = ctx.saved_tensors
        xs = saved[:ns]
        acts = list(saved[ns:ns + nl - 1])
        z = saved[ns + nl - 1]
        relu = chain.act == L.ACT["relu"]
        pres = [] if relu else list(saved[len(saved) - (nl - 1):])
        gy = _c(gy)
        dev = gy.device
        pgrads = []
        # LayerNorm
        if chain.ln is not None:
            mean, rstd = saved[ns + nl], saved[ns + nl + 1]
            g, bt = chain.ln
            n = z.shape[1]
            dz = torch.empty_like(z)
            dg = torch.empty(n, dtype=F64, device=dev)
            db_ = torch.empty(n, dtype=F64, device=dev)
            lib = L.lib()
            scratch = torch.empty(max(int(lib.agn_f64_layernorm_bwd_scratch_bytes(rows, n)) // 8, 1), dtype=F64,
                                  device=dev)
            check(lib.agn_f64_layernorm_bwd(rows, n, ptr(gy), gy.stride(0), ptr(z), z.stride(0), ptr(mean),
                                            ptr(rstd), ptr(g), ptr(dz), dz.stride(0), ptr(dg), ptr(db_),
                                            ptr(scratch), stream()), "f64_layernorm_bwd")
            ln_grads = [dg, db_]
        else:
            dz = gy
            ln_grads = []
        lin_grads = [None] * nl
        for l in range(nl - 1, -1, -1):
            w, b = chain.lins[l]
            dw = torch.empty_like(w)
            dbias = torch.empty(w.shape[0], dtype=F64, device=dev) if b is not None else None
            if l > 0:
                a_in = acts[l - 1]
                wgrad(dz, a_in, None, dw, dbias)
                d_in = torch.empty(rows, w.shape[1], dtype=F64, device=dev)
                # the activation's backward: ReLU on the saved activation, d(pre) = (dz W) . [a_in > 0];
                # others at the saved pre-activation, d(pre) = (dz W) . f'(pre)
                if relu:
                    gemm(rows, w.shape[1], [(dz, None, w.shape[0], w, 0)], d_in, mask=a_in)
                else:
                    gemm(rows, w.shape[1], [(dz, None, w.shape[0], w, 0)], d_in, mask=pres[l - 1],
                         mask_act=1 + chain.act)
                lin_grads[l] = (dw, dbias)
                dz = d_in
            else:
                dxs, k0 = [], 0
                for s, (x, idx) in enumerate(zip(xs, idxs)):
                    k = x.shape[1]
                    wgrad(dz, x, idx, dw[:, k0:k0 + k], dbias if s == 0 else None)
                    if ctx.needs_input_grad[1 + s]:
                        d = torch.empty(rows, k, dtype=F64, device=dev)
                        gemm(rows, k, [(dz, None, w.shape[0], w[:, k0:k0 + k], 0)], d)
                        if idx is not None:
                            d = scatter_rows_sum(d, idx, ctx.nsrc[s])
                        dxs.append(d)
                    else:
                        dxs.append(None)
                    k0 += k
                if ns == 0 and dbias is not None:
                    raise NotImplementedError("aerognn float64 chain without input segments")
                lin_grads[0] = (dw, dbias)
        dadds = []
        for q in range(na):
            if not ctx.needs_input_grad[1 + ns + q]:
                dadds.append(None)
            elif add_idx[q] is not None:
                dadds.append(scatter_rows_sum(dz, add_idx[q], ctx.nadd[q]))
            else:
                dadds.append(dz)
        dres = [gy] if has_resid else []
        for w, b in chain.lins:
            pass
        # parameter grads in Chain.params() order
        for (w, b), (dw, dbias) in zip(chain.lins, lin_grads):
            pgrads.append(dw)
            if b is not None:
                pgrads.append(dbias)
        pgrads += ln_grads
        return (None, *dxs, *dadds, *dres, *pgrads)


def _check_f64(chain, ts):
    """Every operand of a float64 chain must be float64 on one device: the agn_f64_* kernels read
    their buffers as doubles, so a float32 weight given a float64 input (a float32 model fed
    torch.from_numpy data) would be read past its end. Raise as torch does for mm's operands."""
    dev = None
    for t in list(ts) + list(chain.params()):
        if t is None:
            continue
        if t.dtype != F64:
            raise TypeError(f"aerognn float64 path: expected all operands and parameters float64, got {t.dtype} "
                            "(mat1 and mat2 must have the same dtype); call model.double() for float64 inputs")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"aerognn float64 path: operands on {dev} and {t.device}")


def run_chain(chain, xs, idxs=None, rows=None, adds=(), add_idx=(), resid=None):
    _check_f64(chain, list(xs) + list(adds) + [resid])
    idxs = list(idxs) if idxs is not None else [None] * len(xs)
    if rows is None:
        rows = xs[0].shape[0] if idxs[0] is None else idxs[0].numel()
    meta = (chain, idxs, list(add_idx), int(rows), resid is not None)
    ts = list(xs) + list(adds) + ([resid] if resid is not None else [])
    return MLP64Fn.apply(meta, *ts, *chain.params())


class SegSum64Fn(torch.autograd.Function):
    """agg[r] = sum (mean) of the CSC rows rowptr[r] .. rowptr[r+1]-1 of e (receiver order)."""

    @staticmethod
    def forward(ctx, e, rowptr, dst, n, mean):
        e = _c(e)
        out = torch.empty(n, e.shape[1], dtype=F64, device=e.device)
        if n:
            segment_sum(n, e.shape[1], rowptr, None, e, out, mean=mean)
        ctx.rowptr, ctx.dst, ctx.mean, ctx.E = rowptr, dst, mean, e.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        de = torch.empty(ctx.E, g.shape[1], dtype=F64, device=g.device)
        if ctx.E:
            gather_rows(ctx.E, g.shape[1], ctx.dst, g, de, cnt_ptr=ctx.rowptr if ctx.mean else None)
        return de, None, None, None, None


# --------------------------------------------------------------------------- module bindings
def _ln_of(mlp_module):
    return (mlp_module.layer_norm.weight, mlp_module.layer_norm.bias) if mlp_module.use_layer_norm else None


def _check_mlp(m):
    if m.activation_fn not in L.ACT:
        raise NotImplementedError(f"aerognn float64 MLP implements activation_fn in {sorted(L.ACT)}")
    if m.training and m.dropout.p > 0:
        raise NotImplementedError("aerognn float64 MLP: dropout > 0 in training is not implemented")


def mlp_chain(m):
    """models/mlp.py MLP -> Chain (the reference's layer list, mlp.py:21-35)."""
    _check_mlp(m)
    return Chain([(l.weight, l.bias) for l in m.layers], _ln_of(m), m.layer_norm.eps if m.use_layer_norm else 1e-5,
                 act=L.ACT[m.activation_fn])


def mlp_forward(m, x, rows=None):
    """models/mlp.py:40-51 (rows: the chain reads x[rows], MLP.forward_rows)."""
    idx = rows.to(torch.int32).contiguous() if rows is not None else None
    return run_chain(mlp_chain(m), [x], [idx])


def edge_chain(eb):
    """EdgeBlockSum (mgnLayer.py:72-105): [W_e (no bias)] + the mlp's Linears + LayerNorm."""
    seq = list(eb.mlp)
    if any(isinstance(s, torch.nn.Module) and not isinstance(s, (torch.nn.Linear, torch.nn.ReLU, torch.nn.LayerNorm))
           for s in seq):
        raise NotImplementedError("aerognn float64 EdgeBlockSum: Linear / ReLU / LayerNorm chains only")
    lins = [m for m in seq if isinstance(m, torch.nn.Linear)]
    lns = [m for m in seq if isinstance(m, torch.nn.LayerNorm)]
    return Chain([(eb.edge_lin, None)] + [(m.weight, m.bias) for m in lins],
                 (lns[0].weight, lns[0].bias) if lns else None, lns[0].eps if lns else 1e-5)


def edge_update(eb, x, e_csc, level, resid=False):
    """EdgeBlock / EdgeBlockSum on a CSC level: the edge MLP output (+ e when resid)."""
    src, dst = level.src, level.dst
    r = e_csc if resid else None
    if hasattr(eb, "edge_lin"):  # sum trick: h0 = W_e e + (W_s x)[src] + (W_d x + b)[dst]
        ps = run_chain(Chain([(eb.src_lin, None)]), [x])
        pd = run_chain(Chain([(eb.dst_lin, eb.bias)]), [x])
        return run_chain(edge_chain(eb), [e_csc], adds=[ps, pd], add_idx=[src, dst], resid=r)
    # concat: mlp(cat[e, x[src], x[dst]])
    return run_chain(mlp_chain(eb.mlp), [e_csc, x, x], [None, src, dst], rows=e_csc.shape[0], resid=r)


def node_update(nb, x, e_csc, level, resid=False):
    """NodeBlock (mgnLayer.py:132-153): mlp(cat[x, scatter_{add,mean}(e, dst)]) (+ x)."""
    if nb.aggregation not in ("mean", "add"):
        raise ValueError(f"Unsupported aggregation method: {nb.aggregation}")
    agg = SegSum64Fn.apply(e_csc, level.rowptr, level.dst, x.shape[0], nb.aggregation == "mean")
    return run_chain(mlp_chain(nb.mlp), [x, agg], resid=x if resid else None)


def gmp_layer(layer, x, e_csc, level):
    """MeshGraphNetLayer.forward (mgnLayer.py:177-213) on a CSC level: e' = e + Edge, x' = x + Node."""
    require_device(x, e_csc)
    e_new = edge_update(layer.edge_block, x, e_csc, level, resid=True)
    x_new = node_update(layer.node_block, x, e_new, level, resid=True)
    return x_new, e_new
