"""autograd.Functions over the libaerognn kernels: one per reference block.

  MLPFn        models/mlp.py:40-51 (encoders, decoder, any MLP)
  GMPFn        models/mgnLayer.py:177-213 (EdgeBlockSum / EdgeBlock + NodeBlock + residuals)
  PoolNodeFn   bsms_mgn.py:265-267 scatter_mean of node latents (and pos)
  PoolEdgeFn   bsms_mgn.py:283     scatter_mean of edge latents over coalesced edges
  UnpoolFn     bsms_mgn.py:199-200,303-306 coarse[f2c] + skip
  GradBox/SkipFn  skip-gradient side channel of the U-Net (no autograd adds)
  GatherRowsFn / UnpoolRowsFn / WECFn / WECGivenFn  the stale BSMS-GNN ops:
               x[node_indices], Unpool, WeightedEdgeConv with computed / given weights

Forward kernels write the activations the backward needs (relu outputs, pre-LN outputs and
LN statistics); backward kernels run the chain rule per row on MFMA and the weight
gradients are G^T X products accumulated in fp32.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from ._lib import check, ptr
from . import core as _core
from .core import (Pack, WGrad, alg8d_edge, alg8d_node, with_alg, edge_bwd_fused, fused_edge_train_ok, bwd_nblocks,
                   edge32_ok, edge_saves_ok, edge_forward,
                   cost_edge_bwd_fused,
                   proj_kernel_ok, proj_forward, proj_backward, tiled_empty, relu_mask_empty, colsum_rows, cost_edge_bwd, cost_edge_bwd_cat, cost_edge_fwd,
                   cost_edge_fwd_cat, cost_node_bwd, cost_node_fwd, cost_proj, cost_wec_bwd, cost_wec_fwd, dt_code,
                   timed, gather_rows, mlp_backward, mlp_forward, require_device,
                   scatter_rows, segment_max, segment_max_backward, segment_sum, segment_sum2, stream)


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _ln_grads(partial, nblk, M, dtype):
    out = torch.empty(2 * M, dtype=torch.float32, device=partial.device)
    colsum_rows(partial, nblk, 2 * M, out)
    return out[:M].to(dtype), out[M:].to(dtype)


# --------------------------------------------------------------------------- chain specs
class ChainSpec:
    """A Linear/activation chain + optional LayerNorm, bound to nn.Parameters.

    linears: list of (weight, bias_or_None) in order; ln: (gamma, beta) or None.
    Pack keys: W{l} (A = W_l), T{l} (A = W_l^T), b{l}, ln_g, ln_b.
    """

    def __init__(self, linears, ln, hidden, pack: Pack, prefix="", act="relu"):
        if act not in L.ACT:
            raise NotImplementedError(f"aerognn MLP kernels implement activation_fn in {sorted(L.ACT)}, got {act!r}")
        self.act = L.ACT[act]  # AGN_ACT_* between the Linears (mlp.py:37)
        self.linears = linears
        self.ln = ln
        self.hidden = hidden
        self.nlin = len(linears)
        self.in_dim = linears[0][0].shape[1]
        self.out_dim = linears[-1][0].shape[0]
        # training saves (ReLU outputs, pre-LN output) go to the AGN_TILED layout when hidden-wide
        # (agn_wgrad reads tiled operands of width 128 = the production hidden size)
        self.tiled_saves = hidden == 128 and (ln is None or self.out_dim == hidden)
        self.p = prefix
        for l, (w, b) in enumerate(linears):
            M, K = w.shape
            pack.matrix(prefix + f"W{l}", M, K, [(w, 0, 0, False)])
            pack.matrix(prefix + f"T{l}", K, M, [(w, 0, 0, True)])
            if b is not None:
                pack.vector(prefix + f"b{l}", M, [(b, 0)])
        if ln is not None:
            pack.vector(prefix + "ln_g", ln[0].numel(), [(ln[0], 0)])
            pack.vector(prefix + "ln_b", ln[1].numel(), [(ln[1], 0)])
        self.pack = pack

    def wpk(self):
        return [self.pack[self.p + f"W{l}"] for l in range(self.nlin)]

    def wtpk(self):
        return [self.pack[self.p + f"T{l}"] for l in range(self.nlin)]

    def biases(self):
        return [self.pack[self.p + f"b{l}"] if self.linears[l][1] is not None else None for l in range(self.nlin)]

    def lnp(self):
        return (self.pack[self.p + "ln_g"], self.pack[self.p + "ln_b"]) if self.ln is not None else None

    def params(self):
        out = []
        for w, b in self.linears:
            out.append(w)
            if b is not None:
                out.append(b)
        if self.ln is not None:
            out += [self.ln[0], self.ln[1]]
        return out

    def check_hidden(self):
        H = self.hidden
        for l, (w, b) in enumerate(self.linears):
            M, K = w.shape
            if l < self.nlin - 1 and M != H:
                raise NotImplementedError(f"aerognn MLP kernels need every hidden width == {H}, got {M}")
            if l > 0 and K != H:
                raise NotImplementedError(f"aerognn MLP kernels need every hidden width == {H}, got {K}")


def _alloc_saves(spec, rows, dtype, dev, train):
    if not train:
        return None, None, None
    emp = tiled_empty if spec.tiled_saves else (lambda r, w, dt, d: torch.empty(r, w, dtype=dt, device=d))
    acts = [emp(rows, spec.hidden, dtype, dev) for _ in range(spec.nlin - 1)]
    for t in acts:  # what the activation's backward reads; the rows themselves stay for agn_wgrad
        if spec.act == L.ACT["relu"]:
            t.agn_mask = relu_mask_empty(rows, spec.hidden, dev)  # sign bits (AGN_RELU_MASK)
        else:
            t.agn_pre = emp(rows, spec.hidden, dtype, dev)  # the pre-activation (agn_mlp_fwd_args.pre)
    hpre = stats = None
    if spec.ln is not None:
        hpre = emp(rows, spec.out_dim, dtype, dev)
        stats = torch.empty(rows, 2, dtype=torch.float32, device=dev)
    return acts, hpre, stats


def _alloc_gpre(spec, rows, dtype, dev, rowmajor=()):
    """Pre-activation gradient buffers: AGN_TILED when hidden-wide (read only by agn_wgrad), row
    major for layers listed in `rowmajor` (consumed by other kernels) or narrower than hidden."""
    out = []
    for l in range(spec.nlin):
        w = spec.hidden if l < spec.nlin - 1 else spec.out_dim
        if w == spec.hidden == 128 and l not in rowmajor:
            out.append(tiled_empty(rows, w, dtype, dev))
        else:
            out.append(torch.empty(rows, w, dtype=dtype, device=dev))
    return out


def _chain_param_grads(spec, gpre, inputs0, acts, lnp_partial, nblk, wg=None, tag="wgrad_enc"):
    """Grads (in spec.params() order) from stored pre-activation grads.

    Queues the dW/db products on `wg` (a core.WGrad); the returned fp32 tensors are filled
    when wg.run() executes (run here if no batch object is passed in).
    """
    own = wg is None
    wg = wg or WGrad(tag)
    grads = []
    dev = gpre[0].device
    for l, (w, b) in enumerate(spec.linears):
        G = gpre[l]
        M, K = w.shape
        dw = torch.empty(M, K, dtype=torch.float32, device=dev)
        db = torch.empty(M, dtype=torch.float32, device=dev) if b is not None else None
        if l == 0 and isinstance(inputs0, (list, tuple)):
            # column blocks of dW; an (X, idx) block is the gathered operand X[idx] (agn_wgrad's xidx)
            k0 = 0
            for j, X in enumerate(inputs0):
                X, xi = X if isinstance(X, tuple) else (X, None)
                wg.add(G, X, dw[:, k0:k0 + X.shape[1]], db if j == 0 else None, xidx=xi)
                k0 += X.shape[1]
        else:
            wg.add(G, inputs0 if l == 0 else acts[l - 1], dw, db)
        grads.append((dw, w.dtype))
        if b is not None:
            grads.append((db, b.dtype))
    if own:
        wg.run()
    out = [g if g.dtype == dt else g.to(dt) for g, dt in grads]
    if spec.ln is not None:
        g, bb = _ln_grads(lnp_partial, nblk, spec.out_dim, spec.ln[0].dtype)
        out += [g, bb]
    return out


# --------------------------------------------------------------------------- MLP
def _ksegs(x, H):
    """Split an input row of K features into segments of <= H (multiples of 32 but the last)."""
    K = x.shape[1]
    segs, k0 = [], 0
    while k0 < K:
        k = min(H, K - k0)
        segs.append((k0, k))
        k0 += k
    return segs


class MLPFn(torch.autograd.Function):
    """models/mlp.py:40-51. `rows` (int64 / int32 [R] or None): the chain runs on x[rows] with the
    gather done by the kernel's input loads (SEG_GATHER); the input gradient is then scattered
    back with a fixed-order segment sum over the rows that read each input row."""

    @staticmethod
    def forward(ctx, x, spec: ChainSpec, train, rows, *params):
        require_device(x)
        x = _c(x)
        nrow = x.shape[0] if rows is None else rows.numel()
        dt = x.dtype
        out = torch.empty(nrow, spec.out_dim, dtype=dt, device=x.device)
        # an encoder whose input needs no gradient trains on the fused backward (the forward saves nothing)
        fused = train and _core.encoder_fused_ok(spec, dt, x.shape[1], nrow, ctx.needs_input_grad[0])
        acts, hpre, stats = _alloc_saves(spec, nrow, dt, x.device, train and not fused)
        ks = _ksegs(x, spec.hidden)
        if len(ks) > L.MAX_SEG:
            raise NotImplementedError("aerognn MLP input wider than 3 x hidden")
        idx = None
        if rows is not None:
            idx = rows.to(torch.int32).contiguous()
            segs = [(L.SEG_GATHER, k, x.stride(0), x[:, k0:], idx, None) for k0, k in ks]
        else:
            segs = [(L.SEG_PLAIN, k, x.stride(0), x[:, k0:], None, None) for k0, k in ks]
        mlp_forward(rows=nrow, dtype=dt, hidden=spec.hidden, nlin=spec.nlin, act_fn=spec.act, out_dim=spec.out_dim,
                    segs=segs, wpk=spec.wpk(), bias=spec.biases(), ln=spec.lnp(), out=out,
                    acts=acts, hpre=hpre, stats=stats)
        ctx.spec, ctx.idx, ctx.nrow, ctx.fused = spec, idx, nrow, fused
        ctx.acts, ctx.hpre, ctx.stats = acts, hpre, stats
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        spec = ctx.spec
        gy = _c(gy)
        rows = ctx.nrow
        dt = x.dtype
        if ctx.fused:
            # one launch: forward recompute, LayerNorm backward, chain rule, dW1..dW3 / db1..db3 on chip;
            # dW0 / db0 from G0 and the (gathered) input rows on agn_wgrad
            H = spec.hidden
            g0 = torch.empty(rows, H, dtype=dt, device=x.device)
            s_el = x.element_size()
            dW13, db13, part, nblk = _core.encoder_bwd_fused(
                rows=rows, wpk=spec.wpk(), bias=spec.biases(), ln_g=spec.lnp()[0], x=x, xidx=ctx.idx, g=gy, g0=g0,
                tag="enc_bwd", cost=(0.0, 2.0 * rows * H * H * 9, rows * (3 * H * s_el + 2 * x.shape[1] + 4)))
            w0, b0 = spec.linears[0]
            dw0 = torch.empty(w0.shape, dtype=torch.float32, device=x.device)
            db0 = torch.empty(H, dtype=torch.float32, device=x.device) if b0 is not None else None
            wg = WGrad("wgrad_enc")
            wg.add(g0, x, dw0, db0, xidx=ctx.idx)
            wg.run()
            grads = [dw0] + ([db0] if b0 is not None else [])
            for l in range(3):
                w, b = spec.linears[l + 1]
                grads.append(dW13[l])
                if b is not None:
                    grads.append(db13[l])
            grads += list(_ln_grads(part, nblk, H, torch.float32))
            params = spec.params()
            grads = [gr if gr.dtype == p.dtype else gr.to(p.dtype) for gr, p in zip(grads, params)]
            return (None, None, None, None, *grads)
        gpre = _alloc_gpre(spec, rows, dt, x.device)
        ks = _ksegs(x, spec.hidden)
        need_dx = ctx.needs_input_grad[0]
        dparts = [torch.empty(rows, k, dtype=dt, device=x.device) if need_dx else None for _, k in ks]
        nblk = bwd_nblocks(rows)
        part = torch.empty(nblk, 2 * spec.out_dim, dtype=torch.float32, device=x.device) if spec.ln else None
        nblk = mlp_backward(rows=rows, dtype=dt, hidden=spec.hidden, nlin=spec.nlin, act_fn=spec.act, out_dim=spec.out_dim,
                            in_dim=spec.in_dim, wtpk=spec.wtpk(), acts=ctx.acts or [], g=gy, gpre=gpre,
                            ln_g=spec.lnp()[0] if spec.ln else None, hpre=ctx.hpre, stats=ctx.stats,
                            din=[(k, d, False) for (_, k), d in zip(ks, dparts)], ln_partial=part)
        dx = None
        if need_dx:
            dx = dparts[0] if len(dparts) == 1 else torch.cat(dparts, 1)
            if ctx.idx is not None:  # d x[r] = sum over the output rows i with rows[i] = r
                from .graph import group_by
                perm, rp = group_by(ctx.idx, x.shape[0])
                dxs = torch.empty(x.shape[0], x.shape[1], dtype=dt, device=x.device)
                segment_sum(x.shape[0], x.shape[1], rp, perm, dx, dxs)
                dx = dxs
        x0 = x if ctx.idx is None else [(x, ctx.idx)]  # the gathered rows, read through agn_wgrad's xidx
        grads = _chain_param_grads(spec, gpre, x0, ctx.acts, part, nblk)
        return (dx, None, None, None, *grads)


class PermuteRowsFn(torch.autograd.Function):
    """y = x[perm] for a permutation of rows (caller edge order <-> CSC order of a level): a row
    gather on agn_gather_rows both ways (the backward gathers by the inverse permutation)."""

    @staticmethod
    def forward(ctx, x, perm32, inv32):
        require_device(x)
        if x.dim() != 2 or x.shape[0] != perm32.numel() or perm32.numel() != inv32.numel():
            # the gather kernel trusts its index: a row-count mismatch would read past the buffers
            raise ValueError(f"edge rows: got a tensor of shape {tuple(x.shape)} for a level with "
                             f"E = {perm32.numel()} edges (expected [E, features])")
        x = _c(x)
        ctx.inv32 = inv32
        return gather_rows(x.shape[0], x.shape[1], perm32, x, torch.empty_like(x))

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        return gather_rows(g.shape[0], g.shape[1], ctx.inv32, g, torch.empty_like(g)), None, None


def permute_rows(x, perm32, inv32):
    return PermuteRowsFn.apply(x, perm32, inv32)


def to_csc(x, lv):
    """Rows in the caller's edge order -> the level's CSC order (x[lv.perm])."""
    return PermuteRowsFn.apply(x, lv.perm32, lv.inv32)


def from_csc(x, lv):
    """Rows in the level's CSC order -> the caller's edge order (x[lv.perm_inv])."""
    return PermuteRowsFn.apply(x, lv.inv32, lv.perm32)


# --------------------------------------------------------------------------- GMP layer
class LayerSpec:
    """Binds reference blocks (mgnLayer.py:10-213) to packed operands.

    Either block may be None (standalone EdgeBlock / EdgeBlockSum / NodeBlock forwards).
    """

    def __init__(self, edge_block=None, node_block=None):
        self.pack = Pack()
        self.edge = self.node = None
        self.trick = False
        self.gmp_order = False  # GMP (bistride_ops @235) concatenates [x_src, x_dst, e]
        self.aggregation = "add"
        H = None
        if node_block is not None:
            nbm = node_block.mlp
            self.aggregation = node_block.aggregation
            if self.aggregation not in ("add", "mean"):
                raise ValueError(f"Unsupported aggregation method: {self.aggregation}")  # mgnLayer.py:147-148
            H = nbm.layers[0].weight.shape[0]
            self.node = ChainSpec([(m.weight, m.bias) for m in nbm.layers],
                                  (nbm.layer_norm.weight, nbm.layer_norm.bias) if nbm.use_layer_norm else None,
                                  H, self.pack, "n", act=nbm.activation_fn)
        if edge_block is not None:
            eb = edge_block
            self.trick = hasattr(eb, "edge_lin")
            if self.trick:
                seq = list(eb.mlp)
                lins = [m for m in seq if isinstance(m, torch.nn.Linear)]
                lns = [m for m in seq if isinstance(m, torch.nn.LayerNorm)]
                He = eb.edge_lin.shape[0]
                H = He if H is None else H
                self.edge = ChainSpec([(eb.edge_lin, None)] + [(m.weight, m.bias) for m in lins],
                                      (lns[0].weight, lns[0].bias) if lns else None, H, self.pack, "e")
                node_dim = eb.src_lin.shape[1]
                self.pack.matrix("proj", 2 * H, node_dim, [(eb.src_lin, 0, 0, False), (eb.dst_lin, H, 0, False)])
                self.pack.matrix("projT", node_dim, 2 * H, [(eb.src_lin, 0, 0, True), (eb.dst_lin, 0, H, True)])
                self.pack.vector("proj_b", 2 * H, [(eb.bias, H)])
                self.eb = eb
                if He != H or eb.src_lin.shape[0] != H:
                    raise NotImplementedError("aerognn: edge and node hidden widths must match")
            else:
                em = eb.mlp
                H = em.layers[0].weight.shape[0] if H is None else H
                self.edge = ChainSpec([(m.weight, m.bias) for m in em.layers],
                                      (em.layer_norm.weight, em.layer_norm.bias) if em.use_layer_norm else None,
                                      H, self.pack, "e", act=em.activation_fn)
            # (EdgeBlockSum's chain is ReLU whatever activation_fn says: mgnLayer.py:81)
        self.H = H
        if H not in (32, 64, 128):
            raise NotImplementedError(f"aerognn kernels support hidden 32/64/128, got {H}")
        for c in (self.edge, self.node):
            if c is not None:
                c.check_hidden()
                if c.out_dim != H:
                    raise NotImplementedError("aerognn GMP kernels need node_dim == edge_dim == hidden_dim")
        if self.node is not None and self.node.in_dim != 2 * H:
            raise NotImplementedError("aerognn GMP kernels need node_dim == edge_dim == hidden_dim")

    @classmethod
    def from_gmp(cls, gmp):
        """GMP of the stale BSMS-GNN design (bistride_ops @216-250): edge_mlp / node_mlp =
        Sequential(Linear, act, Linear, LayerNorm), edge input cat[x_src, x_dst, e]."""
        self = cls.__new__(cls)
        self.pack = Pack()
        self.trick, self.gmp_order, self.aggregation = False, True, "add"
        acts = {torch.nn.ReLU: "relu", torch.nn.SiLU: "silu", torch.nn.GELU: "gelu", torch.nn.Tanh: "tanh"}
        ea, na = acts.get(type(gmp.edge_mlp[1])), acts.get(type(gmp.node_mlp[1]))
        # the kernels compute the exact (erf) GELU: a tanh-approximated one on either MLP is refused
        tanh_gelu = any(isinstance(m[1], torch.nn.GELU) and m[1].approximate != "none"
                        for m in (gmp.edge_mlp, gmp.node_mlp))
        if ea is None or na is None or tanh_gelu:
            raise NotImplementedError("aerognn GMP kernels implement ReLU / SiLU / GELU / Tanh MLPs")
        e0, e2, eln = gmp.edge_mlp[0], gmp.edge_mlp[2], gmp.edge_mlp[3]
        n0, n2, nln = gmp.node_mlp[0], gmp.node_mlp[2], gmp.node_mlp[3]
        H = e0.weight.shape[0]
        if H not in (32, 64, 128):
            raise NotImplementedError(f"aerognn kernels support hidden 32/64/128, got {H}")
        self.edge = ChainSpec([(e0.weight, e0.bias), (e2.weight, e2.bias)], (eln.weight, eln.bias), H, self.pack, "e",
                              act=ea)
        self.node = ChainSpec([(n0.weight, n0.bias), (n2.weight, n2.bias)], (nln.weight, nln.bias), H, self.pack, "n",
                              act=na)
        self.H = H
        for c in (self.edge, self.node):
            c.check_hidden()
            if c.out_dim != H:
                raise NotImplementedError("aerognn GMP kernels need node_dim == edge_dim == hidden_dim")
        if self.node.in_dim != 2 * H or self.edge.in_dim != 3 * H:
            raise NotImplementedError("aerognn GMP kernels need node_dim == edge_dim == hidden_dim")
        return self

    def edge_params(self):
        if self.edge is None:
            return []
        if self.trick:
            eb = self.eb
            return [eb.edge_lin, eb.src_lin, eb.dst_lin, eb.bias] + self.edge.params()[1:]
        return self.edge.params()

    def node_params(self):
        return self.node.params() if self.node is not None else []

    def params(self):
        return self.edge_params() + self.node_params()


class GMPFn(torch.autograd.Function):
    """x' = x + Node(x, sum_col e'), e' = e + Edge(e, x) on a CSC-ordered level."""

    @staticmethod
    def forward(ctx, x, e, level, spec: LayerSpec, train, *params):
        require_device(x, e)
        x, e = _c(x), _c(e)
        dt, dev = x.dtype, x.device
        N, E, H = x.shape[0], e.shape[0], spec.H
        es, ns = spec.edge, spec.node
        e_out = torch.empty_like(e)
        x_out = torch.empty_like(x)
        # fused edge backward: the chain is recomputed there from the forward's a1 and LayerNorm
        # statistics (or from e and P); the split path's saves are not needed
        fused = train and spec.trick and fused_edge_train_ok(E, dt, H, es.nlin, es.ln is not None)
        # the 32-row-tile forward (agn_edge_forward32, bitwise the resident agn_mlp_forward kernel
        # the fused backward recomputes): inference and the fused training step
        e32 = (spec.trick and (fused or not train) and edge32_ok(dt, H, es.nlin, es.ln is not None, es.act)
               and e.stride(0) == H)
        # fused training on it: the forward saves a1 and the LayerNorm statistics, and the fused
        # backward starts its recompute from them (AEROGNN_EB_SAVED=0: it recomputes from e, P)
        saved = fused and e32 and edge_saves_ok()
        a1s = tiled_empty(E, H, dt, dev) if saved else None
        sts = torch.empty(E, 2, dtype=torch.float32, device=dev) if saved else None
        ea, ehp, est = _alloc_saves(es, E, dt, dev, train and not fused)
        na, nhp, nst = _alloc_saves(ns, N, dt, dev, train)
        P = None
        if spec.trick:
            P = torch.empty(N, 2 * H, dtype=dt, device=dev)
            sz = x.element_size()
            if proj_kernel_ok(x, H):
                proj_forward(N, x, spec.pack["proj"], spec.pack["proj_b"], P,
                             tag="proj", cost=with_alg(alg8d_node(N, H, sz), cost_proj(N, H, sz)))
            else:
                mlp_forward(rows=N, dtype=dt, hidden=H, nlin=1, out_dim=2 * H,
                            segs=[(L.SEG_PLAIN, x.shape[1], x.stride(0), x, None, None)],
                            wpk=[spec.pack["proj"]], bias=[spec.pack["proj_b"]], out=P,
                            tag="proj", cost=with_alg(alg8d_node(N, H, sz), cost_proj(N, H, sz)))
            if e32:
                edge_forward(rows=E, wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), e=e, proj=P, src=level.src,
                             dst=level.dst, out=e_out, a1=a1s, stats=sts,
                             tag="edge_fwd", cost=with_alg(alg8d_edge(E, N, H, sz), cost_edge_fwd(E, N, H, sz, es.nlin,
                                                                                                 False, a1_saves=saved)))
            else:
                mlp_forward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, act_fn=es.act, out_dim=H,
                            segs=[(L.SEG_PLAIN, H, e.stride(0), e, None, None)],
                            wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), proj=P, src=level.src, dst=level.dst,
                            resid=e, out=e_out, acts=ea, hpre=ehp, stats=est,
                            tag="edge_fwd", cost=with_alg(alg8d_edge(E, N, H, sz), cost_edge_fwd(E, N, H, sz, es.nlin,
                                                                                                train and not fused)))
        else:
            se = (L.SEG_PLAIN, H, e.stride(0), e, None, None)
            ss = (L.SEG_GATHER, H, x.stride(0), x, level.src, None)
            sd = (L.SEG_GATHER, H, x.stride(0), x, level.dst, None)
            mlp_forward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, act_fn=es.act, out_dim=H,
                        segs=[ss, sd, se] if spec.gmp_order else [se, ss, sd],
                        wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), resid=e, out=e_out,
                        acts=ea, hpre=ehp, stats=est,
                        tag="edge_fwd", cost=with_alg(alg8d_edge(E, N, H, x.element_size()),
                                                       cost_edge_fwd_cat(E, N, H, x.element_size(), es.nlin, train)))
        # receiver aggregation (mgnLayer.py:144-146): the node kernel's SUM / MEAN input segment
        # walks each receiver's CSC range in edge order (torch_scatter's fp32 order); in training it
        # also stores the sums for the backward. (A separate segment-sum launch and sums fused into
        # the edge kernel were measured slower: DESIGN.md §9, round 3.)
        kind = L.SEG_MEAN if spec.aggregation == "mean" else L.SEG_SUM
        agg = torch.empty(N, H, dtype=dt, device=dev) if train else None
        aseg = (kind, H, e_out.stride(0), e_out, level.rowptr, agg)
        mlp_forward(rows=N, dtype=dt, hidden=H, nlin=ns.nlin, act_fn=ns.act, out_dim=H,
                    segs=[(L.SEG_PLAIN, H, x.stride(0), x, None, None), aseg],
                    wpk=ns.wpk(), bias=ns.biases(), ln=ns.lnp(), resid=x, out=x_out,
                    acts=na, hpre=nhp, stats=nst,
                    tag="node_fwd", cost=with_alg(alg8d_node(N, H, x.element_size()),
                                                   cost_node_fwd(E, N, H, x.element_size(),
                                                                 ns.nlin, train)))
        ctx.spec, ctx.level = spec, level
        ctx.saves = (ea, ehp, est, na, nhp, nst, agg)
        ctx.fused, ctx.proj, ctx.esaves = fused, (P if fused and not saved else None), (a1s, sts)
        ctx.save_for_backward(x, e)
        # an unused e' (the U-Net restores fine edges from the skip, bsms_mgn.py:203) arrives as
        # None instead of a materialised [E,H] zero tensor; the kernels read it as zero
        ctx.set_materialize_grads(False)
        return x_out, e_out

    @staticmethod
    def backward(ctx, gx, ge):
        x, e = ctx.saved_tensors
        spec, lv = ctx.spec, ctx.level
        ea, ehp, est, na, nhp, nst, agg = ctx.saves
        es, ns = spec.edge, spec.node
        dt, dev = x.dtype, x.device
        N, E, H = x.shape[0], e.shape[0], spec.H
        gx = _c(gx) if gx is not None else torch.zeros_like(x)
        ge = _c(ge) if ge is not None else None
        # ---- NodeBlock: d(x), d(agg)
        gpre_n = _alloc_gpre(ns, N, dt, dev)
        dx = torch.empty_like(x)
        dagg = torch.empty(N, H, dtype=dt, device=dev)
        nb_n = bwd_nblocks(N)
        part_n = torch.empty(nb_n, 2 * H, dtype=torch.float32, device=dev) if ns.ln else None
        nb_n = mlp_backward(rows=N, dtype=dt, hidden=H, nlin=ns.nlin, act_fn=ns.act, out_dim=H, in_dim=2 * H, wtpk=ns.wtpk(),
                     acts=na, g=gx, gpre=gpre_n, ln_g=ns.lnp()[0] if ns.ln else None, hpre=nhp, stats=nst,
                     din=[(H, dx, True), (H, dagg, False)], ln_partial=part_n,
                     tag="node_bwd", cost=with_alg(alg8d_node(N, H, x.element_size(), bwd=True, proj=spec.trick),
                                                   cost_node_bwd(N, H, x.element_size(), ns.nlin)))
        if spec.aggregation == "mean":  # scatter_mean backward: / max(deg, 1)
            dagg = gather_rows(N, H, None, dagg, torch.empty_like(dagg), cnt_ptr=lv.rowptr)
        # ---- EdgeBlock: d(e) (+ residual), pre-activation grads
        fused = ctx.fused
        de = torch.empty_like(e)
        sz = x.element_size()
        if fused:
            # one launch: forward recompute, LayerNorm backward, chain rule, dW1..dW3 / db1..db3
            g0 = torch.empty(E, H, dtype=dt, device=dev)
            a1s, sts = ctx.esaves
            dW13, db13, part_e, nb_e = edge_bwd_fused(
                rows=E, wpk=es.wpk(), wtpk0=es.wtpk()[0], bias=es.biases(), ln_g=es.lnp()[0], e=e, proj=ctx.proj, src=lv.src, dst=lv.dst,
                g=ge, g2=dagg, de=de, g0=g0, tag="edge_bwd", a1=a1s, stats=sts,
                cost=with_alg(alg8d_edge(E, N, H, sz, bwd=True), cost_edge_bwd_fused(E, N, H, sz, saved=a1s is not None)))
        else:
            nb_e = bwd_nblocks(E)
            part_e = torch.empty(nb_e, 2 * H, dtype=torch.float32, device=dev) if es.ln else None
            gpre_e = _alloc_gpre(es, E, dt, dev, rowmajor=(0,) if spec.trick else ())
            if spec.trick:
                din = [(H, de, True)]
            else:
                dxs = torch.empty(E, H, dtype=dt, device=dev)
                dxd = torch.empty(E, H, dtype=dt, device=dev)
                din = [(H, dxs, False), (H, dxd, False), (H, de, True)] if spec.gmp_order else \
                    [(H, de, True), (H, dxs, False), (H, dxd, False)]
            nb_e = mlp_backward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, act_fn=es.act, out_dim=H, in_dim=es.in_dim,
                                wtpk=es.wtpk(), acts=ea, g=ge, g2=dagg, gidx=lv.dst, gpre=gpre_e,
                                ln_g=es.lnp()[0] if es.ln else None, hpre=ehp, stats=est, din=din, ln_partial=part_e,
                                tag="edge_bwd",
                                cost=with_alg(alg8d_edge(E, N, H, sz, bwd=True),
                                              (cost_edge_bwd if spec.trick else cost_edge_bwd_cat)(E, N, H, sz,
                                                                                                   es.nlin)))
            g0 = gpre_e[0]
        grads_edge = []
        if spec.trick:
            # sum-trick: h0 = e W_e^T + P_s[src] + P_d[dst]: dP by sender / receiver groups
            # (dP_d formed on the fused kernel's dW waves, round 5, measured slower once the chain
            # waves got faster: DESIGN.md §9 round 6)
            dPs = segment_sum(N, H, lv.rowptr_src, lv.perm_src, g0, torch.empty(N, H, dtype=dt, device=dev))
            dPd = segment_sum(N, H, lv.rowptr, None, g0, torch.empty(N, H, dtype=dt, device=dev))
            if proj_kernel_ok(dx, H):
                s_el = dx.element_size()
                proj_backward(N, dPs, dPd, spec.pack["projT"], dx, tag="proj_bwd",
                              cost=with_alg(alg8d_node(N, H, s_el, bwd=True), (4 * N * H * s_el, 4.0 * N * H * H)))
            else:
                mlp_forward(rows=N, dtype=dt, hidden=H, nlin=1, out_dim=H,
                            segs=[(L.SEG_PLAIN, H, H, dPs, None, None), (L.SEG_PLAIN, H, H, dPd, None, None)],
                            wpk=[spec.pack["projT"]], bias=[None], resid=dx, out=dx)
            eb = spec.eb
            # E-row (edge chain) and N-row (projection, node chain) weight gradients go to separate
            # agn_wgrad launches: one split count serves all descs of a launch, and mixing 6x
            # different row counts leaves most workgroups idle behind the edge descs (measured)
            wg = WGrad("wgrad_node")
            if fused:
                dwe = torch.empty(H, H, dtype=torch.float32, device=dev)
                we = WGrad("wgrad_edge")
                we.add(g0, e, dwe)
                we.run()
                eg = [dwe]
                for l in range(3):
                    eg += [dW13[l], db13[l]]
                eg = eg[:1] + [t if t.dtype == p.dtype else t.to(p.dtype) for t, p in zip(eg[1:], es.params()[1:7])]
                eg += list(_ln_grads(part_e, nb_e, H, es.ln[0].dtype))
            else:
                eg = _chain_param_grads(es, gpre_e, e, ea, part_e, nb_e, tag="wgrad_edge")
            dws = torch.empty(H, x.shape[1], dtype=torch.float32, device=dev)
            dwd = torch.empty(H, x.shape[1], dtype=torch.float32, device=dev)
            dbd = torch.empty(H, dtype=torch.float32, device=dev)
            wg.add(dPs, x, dws)
            wg.add(dPd, x, dwd, dbd)
            grads_node = _chain_param_grads(ns, gpre_n, [x, agg], na, part_n, nb_n, wg)
            wg.run()
            if fused and eg[0].dtype != es.linears[0][0].dtype:
                eg[0] = eg[0].to(es.linears[0][0].dtype)
            grads_edge = [eg[0], dws.to(eb.src_lin.dtype), dwd.to(eb.dst_lin.dtype), dbd.to(eb.bias.dtype)] + eg[1:]
            return (dx, de, None, None, None, *grads_edge, *grads_node)
        else:
            # concat edge MLP: dx += scatter_add(d x_src, src) + scatter_add(d x_dst, dst) in one pass
            # (fp32, one rounding), and W_0's x_src / x_dst column blocks from gathered operands
            segment_sum2(N, H, dx, (lv.rowptr_src, lv.perm_src, dxs), (lv.rowptr, None, dxd), dx)
            xs, xd = (x, lv.src), (x, lv.dst)
            grads_edge = _chain_param_grads(es, gpre_e, [xs, xd, e] if spec.gmp_order else [e, xs, xd],
                                            ea, part_e, nb_e, tag="wgrad_edge")
        grads_node = _chain_param_grads(ns, gpre_n, [x, agg], na, part_n, nb_n, tag="wgrad_node")
        return (dx, de, None, None, None, *grads_edge, *grads_node)


# --------------------------------------------------------------------------- pooling
class GradBox:
    """Side channel for a U-Net skip tensor's up-path gradient (bsms_mgn.py:196-206).

    A skip tensor has two consumers: the pooling of the down path and the up path (skip add /
    restored fine edges). Autograd would sum their gradients with a separate [rows, H] add; here
    the up-path consumer parks its gradient in the box (returning None to autograd) and the
    pooling backward — which the graph orders after it — adds it inside its gather kernel.
    """
    __slots__ = ("g", "armed")

    def __init__(self):
        self.g = None
        self.armed = False

    def put(self, g):
        self.g = g if self.g is None else self.g + g

    def take(self):
        if self.armed and self.g is None:
            raise RuntimeError("aerognn: skip gradient missing (autograd order violated)")
        g, self.g = self.g, None
        return g


class SkipFn(torch.autograd.Function):
    """Identity for a skip tensor re-used on the up path; its gradient goes to `box`."""

    @staticmethod
    def forward(ctx, t, box):
        box.armed = True
        ctx.box = box
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        ctx.box.put(g)
        return None, None


class PoolNodeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pool, box=None):
        x = _c(x)
        out = torch.empty(pool.nc, x.shape[1], dtype=x.dtype, device=x.device)
        segment_sum(pool.nc, x.shape[1], pool.c2f_ptr, pool.c2f, x, out, mean=True)
        ctx.pool, ctx.box = pool, box
        ctx.n = x.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        p = ctx.pool
        g = _c(g)
        add = ctx.box.take() if ctx.box is not None else None
        dx = torch.empty(ctx.n, g.shape[1], dtype=g.dtype, device=g.device)
        gather_rows(ctx.n, g.shape[1], p.f2c, g, dx, cnt_ptr=p.c2f_ptr, add=_c(add) if add is not None else None)
        return dx, None, None


class PoolEdgeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, e, pool, box=None):
        e = _c(e)
        ec = pool.coarse.E
        out = torch.empty(ec, e.shape[1], dtype=e.dtype, device=e.device)
        segment_sum(ec, e.shape[1], pool.cmem_ptr, pool.cand_sorted, e, out, mean=True)
        ctx.pool, ctx.box = pool, box
        ctx.n = e.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        p = ctx.pool
        g = _c(g)
        add = ctx.box.take() if ctx.box is not None else None
        de = torch.empty(ctx.n, g.shape[1], dtype=g.dtype, device=g.device)
        gather_rows(ctx.n, g.shape[1], p.inv, g, de, cnt_ptr=p.cmem_ptr, add=_c(add) if add is not None else None)
        return de, None, None


class UnpoolFn(torch.autograd.Function):
    """x_fine = coarse[f2c] + skip (bsms_mgn.py:199-200, 303-306). With `box`, the skip's
    gradient (the identity) is parked for the matching PoolNodeFn backward."""

    @staticmethod
    def forward(ctx, coarse, skip, pool, box=None):
        coarse, skip = _c(coarse), _c(skip)
        n = skip.shape[0]
        out = torch.empty_like(skip)
        gather_rows(n, skip.shape[1], pool.f2c, coarse, out, add=skip)
        ctx.pool, ctx.box = pool, box
        if box is not None:
            box.armed = True
        return out

    @staticmethod
    def backward(ctx, g):
        p = ctx.pool
        g = _c(g)
        dc = torch.empty(p.nc, g.shape[1], dtype=g.dtype, device=g.device)
        segment_sum(p.nc, g.shape[1], p.c2f_ptr, p.c2f, g, dc)
        if ctx.box is not None:
            ctx.box.put(g)
            return dc, None, None, None
        return dc, g, None, None


# --------------------------------------------------------------------------- standalone blocks
class EdgeBlockFn(torch.autograd.Function):
    """EdgeBlockSum / EdgeBlock.forward alone (mgnLayer.py:32-49, 93-105): no residual."""

    @staticmethod
    def forward(ctx, x, e, level, spec: LayerSpec, train, *params):
        require_device(x, e)
        x, e = _c(x), _c(e)
        dt, dev = x.dtype, x.device
        N, E, H = x.shape[0], e.shape[0], spec.H
        es = spec.edge
        out = torch.empty(E, H, dtype=dt, device=dev)
        ea, ehp, est = _alloc_saves(es, E, dt, dev, train)
        if spec.trick:
            P = torch.empty(N, 2 * H, dtype=dt, device=dev)
            mlp_forward(rows=N, dtype=dt, hidden=H, nlin=1, out_dim=2 * H,
                        segs=[(L.SEG_PLAIN, x.shape[1], x.stride(0), x, None, None)],
                        wpk=[spec.pack["proj"]], bias=[spec.pack["proj_b"]], out=P)
            segs = [(L.SEG_PLAIN, H, e.stride(0), e, None, None)]
        else:
            P = None
            segs = [(L.SEG_PLAIN, H, e.stride(0), e, None, None),
                    (L.SEG_GATHER, H, x.stride(0), x, level.src, None),
                    (L.SEG_GATHER, H, x.stride(0), x, level.dst, None)]
        mlp_forward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, act_fn=es.act, out_dim=H, segs=segs, wpk=es.wpk(),
                    bias=es.biases(), ln=es.lnp(), proj=P, src=level.src if P is not None else None,
                    dst=level.dst if P is not None else None, out=out, acts=ea, hpre=ehp, stats=est)
        ctx.spec, ctx.level, ctx.saves = spec, level, (ea, ehp, est)
        ctx.save_for_backward(x, e)
        return out

    @staticmethod
    def backward(ctx, g):
        x, e = ctx.saved_tensors
        spec, lv = ctx.spec, ctx.level
        ea, ehp, est = ctx.saves
        es = spec.edge
        dt, dev = x.dtype, x.device
        N, E, H = x.shape[0], e.shape[0], spec.H
        g = _c(g)
        gpre = _alloc_gpre(es, E, dt, dev, rowmajor=(0,) if spec.trick else ())
        nb = bwd_nblocks(E)
        part = torch.empty(nb, 2 * H, dtype=torch.float32, device=dev) if es.ln else None
        de = torch.empty_like(e)
        if spec.trick:
            din = [(H, de, False)]
        else:
            dxs = torch.empty(E, H, dtype=dt, device=dev)
            dxd = torch.empty(E, H, dtype=dt, device=dev)
            din = [(H, de, False), (H, dxs, False), (H, dxd, False)]
        nb = mlp_backward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, act_fn=es.act, out_dim=H, in_dim=es.in_dim, wtpk=es.wtpk(),
                     acts=ea, g=g, gpre=gpre, ln_g=es.lnp()[0] if es.ln else None, hpre=ehp, stats=est,
                     din=din, ln_partial=part)
        if spec.trick:
            g0 = gpre[0]
            dPs = segment_sum(N, H, lv.rowptr_src, lv.perm_src, g0, torch.empty(N, H, dtype=dt, device=dev))
            dPd = segment_sum(N, H, lv.rowptr, None, g0, torch.empty(N, H, dtype=dt, device=dev))
            dx = torch.zeros_like(x)
            mlp_forward(rows=N, dtype=dt, hidden=H, nlin=1, out_dim=H,
                        segs=[(L.SEG_PLAIN, H, H, dPs, None, None), (L.SEG_PLAIN, H, H, dPd, None, None)],
                        wpk=[spec.pack["projT"]], bias=[None], out=dx)
            eg = _chain_param_grads(es, gpre, e, ea, part, nb, tag="wgrad_edge")
            eb = spec.eb
            wg = WGrad("wgrad_node")
            dws = torch.empty(H, x.shape[1], dtype=torch.float32, device=dev)
            dwd = torch.empty(H, x.shape[1], dtype=torch.float32, device=dev)
            dbd = torch.empty(H, dtype=torch.float32, device=dev)
            wg.add(dPs, x, dws)
            wg.add(dPd, x, dwd, dbd)
            wg.run()
            grads = [eg[0], dws.to(eb.src_lin.dtype), dwd.to(eb.dst_lin.dtype), dbd.to(eb.bias.dtype)] + eg[1:]
        else:
            dx = segment_sum2(N, H, None, (lv.rowptr_src, lv.perm_src, dxs), (lv.rowptr, None, dxd),
                              torch.empty(N, H, dtype=dt, device=dev))
            grads = _chain_param_grads(es, gpre, [e, (x, lv.src), (x, lv.dst)], ea, part, nb, tag="wgrad_edge")
        return (dx, de, None, None, None, *grads)


class NodeBlockFn(torch.autograd.Function):
    """NodeBlock.forward alone (mgnLayer.py:134-153): mlp(cat[x, scatter(e, col)]), no residual."""

    @staticmethod
    def forward(ctx, x, e, level, spec: LayerSpec, train, *params):
        require_device(x, e)
        x, e = _c(x), _c(e)
        dt, dev = x.dtype, x.device
        N, H = x.shape[0], spec.H
        ns = spec.node
        out = torch.empty(N, H, dtype=dt, device=dev)
        na, nhp, nst = _alloc_saves(ns, N, dt, dev, train)
        agg = torch.empty(N, H, dtype=dt, device=dev) if train else None
        kind = L.SEG_MEAN if spec.aggregation == "mean" else L.SEG_SUM
        mlp_forward(rows=N, dtype=dt, hidden=H, nlin=ns.nlin, act_fn=ns.act, out_dim=H,
                    segs=[(L.SEG_PLAIN, H, x.stride(0), x, None, None),
                          (kind, H, e.stride(0), e, level.rowptr, agg)],
                    wpk=ns.wpk(), bias=ns.biases(), ln=ns.lnp(), out=out, acts=na, hpre=nhp, stats=nst)
        ctx.spec, ctx.level, ctx.saves = spec, level, (na, nhp, nst, agg)
        ctx.save_for_backward(x, e)
        return out

    @staticmethod
    def backward(ctx, g):
        x, e = ctx.saved_tensors
        spec, lv = ctx.spec, ctx.level
        na, nhp, nst, agg = ctx.saves
        ns = spec.node
        dt, dev = x.dtype, x.device
        N, E, H = x.shape[0], e.shape[0], spec.H
        g = _c(g)
        gpre = _alloc_gpre(ns, N, dt, dev)
        dx = torch.empty_like(x)
        dagg = torch.empty(N, H, dtype=dt, device=dev)
        nb = bwd_nblocks(N)
        part = torch.empty(nb, 2 * H, dtype=torch.float32, device=dev) if ns.ln else None
        nb = mlp_backward(rows=N, dtype=dt, hidden=H, nlin=ns.nlin, act_fn=ns.act, out_dim=H, in_dim=2 * H, wtpk=ns.wtpk(),
                     acts=na, g=g, gpre=gpre, ln_g=ns.lnp()[0] if ns.ln else None, hpre=nhp, stats=nst,
                     din=[(H, dx, False), (H, dagg, False)], ln_partial=part)
        de = torch.empty_like(e)
        gather_rows(E, H, lv.dst, dagg, de, cnt_ptr=lv.rowptr if spec.aggregation == "mean" else None)
        grads = _chain_param_grads(ns, gpre, [x, agg], na, part, nb, tag="wgrad_node")
        return (dx, de, None, None, None, *grads)


# --------------------------------------------------------------------------- BSMS-GNN (stale design)
class GatherRowsFn(torch.autograd.Function):
    """y = x[idx] (old bsms_mgn @145: x = x[node_indices[i]]); idx unique. Backward scatters."""

    @staticmethod
    def forward(ctx, x, idx32):
        x = _c(x)
        out = torch.empty(idx32.numel(), x.shape[1], dtype=x.dtype, device=x.device)
        gather_rows(idx32.numel(), x.shape[1], idx32, x, out)
        ctx.idx, ctx.n = idx32, x.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        dx = torch.zeros(ctx.n, g.shape[1], dtype=g.dtype, device=g.device)
        scatter_rows(ctx.idx, g, dx)
        return dx, None


class UnpoolRowsFn(torch.autograd.Function):
    """Unpool.forward (bistride_ops @102): zeros[n_fine, C]; x_fine[indices] = x_coarse."""

    @staticmethod
    def forward(ctx, xc, idx32, n_fine):
        xc = _c(xc)
        out = torch.zeros(n_fine, xc.shape[1], dtype=xc.dtype, device=xc.device)
        scatter_rows(idx32, xc, out)
        ctx.idx = idx32
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        dxc = torch.empty(ctx.idx.numel(), g.shape[1], dtype=g.dtype, device=g.device)
        gather_rows(ctx.idx.numel(), g.shape[1], ctx.idx, g, dxc)
        return dxc, None, None


class WecSpec:
    """Packed operands of a WeightedEdgeConv (bistride_ops @136): transform T [out, in] (+b_T),
    edge_weight_mlp = Linear(2 in + 1, 64) -> ReLU -> Linear(64, 1) -> Sigmoid."""

    HID = 64

    def __init__(self, mod):
        T, W1, W2 = mod.transform, mod.edge_weight_mlp[0], mod.edge_weight_mlp[2]
        self.inp, self.out = T.weight.shape[1], T.weight.shape[0]
        i, o, hd = self.inp, self.out, self.HID
        if i not in (32, 64, 128) or o not in (64, 128) or W1.weight.shape[0] != hd:
            raise NotImplementedError("aerognn WeightedEdgeConv: in_dim 32/64/128, out_dim 64/128, hidden 64")
        self.mod = mod
        p = self.pack = Pack()
        p.matrix("T", o, i, [(T.weight, 0, 0, False)])
        p.vector("Tb", o, [(T.bias, 0)])
        p.matrix("W1", 2 * hd, i, [(W1.weight[:, :i], 0, 0, False), (W1.weight[:, i:2 * i], hd, 0, False)])
        p.vector("W1b", 2 * hd, [(W1.bias, hd)])
        p.vector("w1c", hd, [(W1.weight[:, 2 * i], 0)])
        p.vector("w2", hd + 1, [(W2.weight[0], 0), (W2.bias, hd)])
        p.matrix("back", i, o + 2 * hd, [(T.weight, 0, 0, True), (W1.weight[:, :i], 0, o, True),
                                         (W1.weight[:, i:2 * i], 0, o + hd, True)])
        p.matrix("backT", i, o, [(T.weight, 0, 0, True)])

    def params(self):
        m = self.mod
        return [m.edge_weight_mlp[0].weight, m.edge_weight_mlp[0].bias, m.edge_weight_mlp[2].weight,
                m.edge_weight_mlp[2].bias, m.transform.weight, m.transform.bias]


def _wec_args(spec, x, level, mean):
    a = L.WecArgs()
    a.n, a.e, a.dtype = x.shape[0], level.E, dt_code(x.dtype)
    a.out_dim, a.hid, a.mean = spec.out, WecSpec.HID, int(mean)
    a.rowptr, a.src, a.dst, a.perm = ptr(level.rowptr), ptr(level.src), ptr(level.dst), ptr(level.perm)
    a.rowptr_src, a.perm_src = ptr(level.rowptr_src), ptr(level.perm_src)
    return a


def _wec_tx(spec, x):
    tx = torch.empty(x.shape[0], spec.out, dtype=x.dtype, device=x.device)
    mlp_forward(rows=x.shape[0], dtype=x.dtype, hidden=spec.inp, nlin=1, out_dim=spec.out,
                segs=[(L.SEG_PLAIN, spec.inp, x.stride(0), x, None, None)],
                wpk=[spec.pack["T"]], bias=[spec.pack["Tb"]], out=tx)
    return tx


class WECFn(torch.autograd.Function):
    """WeightedEdgeConv with computed weights (bistride_ops @152-210) -> (out, w [E,1])."""

    @staticmethod
    def forward(ctx, x, pos, level, spec, mean, *params):
        require_device(x, pos)
        x = _c(x)
        dt, dev = x.dtype, x.device
        N, E, hd = x.shape[0], level.E, WecSpec.HID
        spec.pack.update(dt, dev)
        pab = torch.empty(N, 2 * hd, dtype=dt, device=dev)
        mlp_forward(rows=N, dtype=dt, hidden=spec.inp, nlin=1, out_dim=2 * hd,
                    segs=[(L.SEG_PLAIN, spec.inp, x.stride(0), x, None, None)],
                    wpk=[spec.pack["W1"]], bias=[spec.pack["W1b"]], out=pab)
        tx = _wec_tx(spec, x)
        pos32 = pos.float().contiguous()
        w = torch.empty(E, 1, dtype=dt, device=dev)
        out = torch.empty(N, spec.out, dtype=dt, device=dev)
        a = _wec_args(spec, x, level, mean)
        a.pos_dim, a.pos_ld, a.pos = pos32.shape[1], pos32.stride(0), ptr(pos32)
        a.pab, a.tx, a.w1c, a.w2 = ptr(pab), ptr(tx), spec.pack["w1c"], spec.pack["w2"]
        a.w_out, a.out = ptr(w), ptr(out)
        with timed("wec_fwd", cost_wec_fwd(E, N, spec.out, x.element_size())):
            check(L.lib().agn_wec_forward(C.byref(a), stream()), "wec_forward")
        ctx.spec, ctx.level, ctx.mean = spec, level, mean
        ctx.save_for_backward(x, pos32, pab, tx)
        ctx.set_materialize_grads(False)
        return out, w

    @staticmethod
    def backward(ctx, dout, dw):
        x, pos32, pab, tx = ctx.saved_tensors
        spec, level = ctx.spec, ctx.level
        dt, dev = x.dtype, x.device
        N, E, hd = x.shape[0], level.E, WecSpec.HID
        if dout is None:
            dout = torch.zeros(N, spec.out, dtype=dt, device=dev)
        dout = _c(dout)
        s_csc = torch.empty(E, dtype=torch.float32, device=dev)
        dh = torch.empty(E, hd, dtype=torch.float32, device=dev)
        dpa = torch.empty(N, hd, dtype=dt, device=dev)
        dpb = torch.empty(N, hd, dtype=dt, device=dev)
        dtx = torch.empty(N, spec.out, dtype=dt, device=dev)
        nblk = int(L.lib().agn_wec_blocks(N))
        partial = torch.empty(max(nblk, 1), 2 * hd + 1, dtype=torch.float32, device=dev)
        a = _wec_args(spec, x, level, ctx.mean)
        a.pos_dim, a.pos_ld, a.pos = pos32.shape[1], pos32.stride(0), ptr(pos32)
        a.pab, a.tx, a.w1c, a.w2 = ptr(pab), ptr(tx), spec.pack["w1c"], spec.pack["w2"]
        dw = _c(dw) if dw is not None else None
        a.dout, a.gw = ptr(dout), ptr(dw)
        a.s_csc, a.dh, a.dpa, a.dpb, a.dtx, a.partial = ptr(s_csc), ptr(dh), ptr(dpa), ptr(dpb), ptr(dtx), ptr(partial)
        with timed("wec_bwd", cost_wec_bwd(E, N, spec.out, x.element_size())):
            check(L.lib().agn_wec_backward(C.byref(a), stream()), "wec_backward")
        i, o = spec.inp, spec.out
        dx = torch.empty_like(x)
        mlp_forward(rows=N, dtype=dt, hidden=i, nlin=1, out_dim=i,
                    segs=[(L.SEG_PLAIN, o, o, dtx, None, None), (L.SEG_PLAIN, hd, hd, dpa, None, None),
                          (L.SEG_PLAIN, hd, hd, dpb, None, None)],
                    wpk=[spec.pack["back"]], bias=[None], out=dx)
        W1 = spec.mod.edge_weight_mlp[0].weight
        dW1 = torch.empty(hd, 2 * i + 1, dtype=torch.float32, device=dev)
        db1 = torch.empty(hd, dtype=torch.float32, device=dev)
        dT = torch.empty(o, i, dtype=torch.float32, device=dev)
        dTb = torch.empty(o, dtype=torch.float32, device=dev)
        wg = WGrad()
        wg.add(dtx, x, dT, dTb)
        wg.add(dpa, x, dW1[:, :i])
        wg.add(dpb, x, dW1[:, i:2 * i], db1)
        wg.run()
        red = torch.empty(2 * hd + 1, dtype=torch.float32, device=dev)
        colsum_rows(partial, nblk, 2 * hd + 1, red)
        dW1[:, 2 * i].copy_(red[hd:2 * hd])
        ps = spec.params()
        grads = [dW1, db1, red[:hd].view(1, hd), red[2 * hd:], dT, dTb]
        grads = [g.to(p.dtype) for g, p in zip(grads, ps)]
        return (dx, None, None, None, None, *grads)


class WECGivenFn(torch.autograd.Function):
    """WeightedEdgeConv with given weights (compute_weights=False, bistride_ops @173)."""

    @staticmethod
    def forward(ctx, x, w, level, spec, mean, *params):
        require_device(x, w)
        x = _c(x)
        dt, dev = x.dtype, x.device
        spec.pack.update(dt, dev)
        w = _c(w.to(dt))
        tx = _wec_tx(spec, x)
        out = torch.empty(x.shape[0], spec.out, dtype=dt, device=dev)
        a = _wec_args(spec, x, level, mean)
        a.tx, a.w_in, a.out = ptr(tx), ptr(w), ptr(out)
        check(L.lib().agn_wec_forward(C.byref(a), stream()), "wec_forward")
        ctx.spec, ctx.level, ctx.mean = spec, level, mean
        ctx.save_for_backward(x, w, tx)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w, tx = ctx.saved_tensors
        spec, level = ctx.spec, ctx.level
        dt, dev = x.dtype, x.device
        N, E = x.shape[0], level.E
        dout = _c(dout)
        s_csc = torch.empty(E, dtype=torch.float32, device=dev)
        dtx = torch.empty(N, spec.out, dtype=dt, device=dev)
        dw = torch.empty(E, 1, dtype=dt, device=dev) if ctx.needs_input_grad[1] else None
        a = _wec_args(spec, x, level, ctx.mean)
        a.tx, a.w_in, a.dout, a.s_csc, a.dtx, a.dw_in = ptr(tx), ptr(w), ptr(dout), ptr(s_csc), ptr(dtx), ptr(dw)
        check(L.lib().agn_wec_backward(C.byref(a), stream()), "wec_backward")
        dx = torch.empty_like(x)
        mlp_forward(rows=N, dtype=dt, hidden=spec.inp, nlin=1, out_dim=spec.inp,
                    segs=[(L.SEG_PLAIN, spec.out, spec.out, dtx, None, None)],
                    wpk=[spec.pack["backT"]], bias=[None], out=dx)
        dT = torch.empty(spec.out, spec.inp, dtype=torch.float32, device=dev)
        dTb = torch.empty(spec.out, dtype=torch.float32, device=dev)
        wg = WGrad()
        wg.add(dtx, x, dT, dTb)
        wg.run()
        T = spec.mod.transform
        return (dx, dw, None, None, None, dT.to(T.weight.dtype), dTb.to(T.bias.dtype))


# --------------------------------------------------------------------------- global pooling
class GraphGroups:
    """Node grouping by graph id for global pooling (poolmgn.py:132-141): `perm`/`rowptr` group the
    nodes of each graph 0..G-1 (stable, any batch order; G = batch.max() + 1 as PyG's global pools
    size it), `bcast` is the row index of the reference's broadcast back to nodes,
    `pooled.repeat_interleave(bincount(batch))` (= batch itself when batch is sorted), `bptr` the
    CSR grouping of `bcast` (contiguous by construction) for the broadcast backward."""

    def __init__(self, batch, n, device):
        from .graph import group_by
        if batch is None:
            self.G = 1
            self.perm = None
            self.rowptr = torch.tensor([0, n], dtype=torch.int32, device=device)
            self.bcast = torch.zeros(n, dtype=torch.int32, device=device)
            self.bptr = self.rowptr
            return
        b32 = batch.to(torch.int32)
        self.G = int(batch.max().item()) + 1 if n > 0 else 0
        self.perm, self.rowptr = group_by(b32, self.G)
        counts = self.rowptr[1:] - self.rowptr[:-1]
        self.bcast = torch.repeat_interleave(torch.arange(self.G, dtype=torch.int32, device=device), counts)
        self.bptr = self.rowptr  # bcast rows of graph g are rowptr[g]..rowptr[g+1]-1


class GlobalPoolFn(torch.autograd.Function):
    """global_{mean,add,max}_pool(x, batch) (torch_geometric; poolmgn.py:38-45) on libaerognn:
    segment sum / mean (fixed member order) or segment max with first-argmax backward."""

    @staticmethod
    def forward(ctx, x, groups, method):
        x = _c(x)
        G, k = groups.G, x.shape[1]
        out = torch.empty(G, k, dtype=x.dtype, device=x.device)
        ctx.groups, ctx.method, ctx.n = groups, method, x.shape[0]
        if method in ("mean", "add"):
            segment_sum(G, k, groups.rowptr, groups.perm, x, out, mean=(method == "mean"))
        elif method == "max":
            arg = torch.empty(G, k, dtype=torch.int32, device=x.device)
            segment_max(G, k, groups.rowptr, groups.perm, x, out, arg)
            ctx.arg = arg
        else:
            raise ValueError(f"Unsupported global pooling method: {method}")
        return out

    @staticmethod
    def backward(ctx, g):
        grp = ctx.groups
        g = _c(g)
        k = g.shape[1]
        if ctx.method == "max":
            dx = torch.zeros(ctx.n, k, dtype=g.dtype, device=g.device)
            segment_max_backward(grp.G, k, ctx.arg, g, dx)
            return dx, None, None
        # d x[i] = g[graph(i)] (/ count for mean): a row gather through the node -> graph map
        node_graph = torch.empty(ctx.n, dtype=torch.int32, device=g.device)
        if grp.perm is None:
            node_graph.zero_()
        else:
            node_graph[grp.perm.long()] = grp.bcast
        dx = torch.empty(ctx.n, k, dtype=g.dtype, device=g.device)
        gather_rows(ctx.n, k, node_graph, g, dx, cnt_ptr=grp.rowptr if ctx.method == "mean" else None)
        return dx, None, None


class BroadcastRowsFn(torch.autograd.Function):
    """pooled.repeat_interleave(bincount(batch), dim=0) (poolmgn.py:134): y[i] = pooled[bcast[i]];
    backward = per-graph segment sum of the row gradients (contiguous groups)."""

    @staticmethod
    def forward(ctx, pooled, groups):
        pooled = _c(pooled)
        n = groups.bcast.numel()
        out = torch.empty(n, pooled.shape[1], dtype=pooled.dtype, device=pooled.device)
        gather_rows(n, pooled.shape[1], groups.bcast, pooled, out)
        ctx.groups, ctx.G = groups, pooled.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        dp = torch.empty(ctx.G, g.shape[1], dtype=g.dtype, device=g.device)
        segment_sum(ctx.G, g.shape[1], ctx.groups.bptr, None, g, dp)
        return dp, None
