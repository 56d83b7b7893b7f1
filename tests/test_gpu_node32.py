"""The node MLP forward with the receiver aggregation walked in (csrc/node32_fwd.hip), which
agn_mlp_forward picks for a processor layer's node MLP without training saves, against the
general kernel (AGN_OPT_RESIDENT = 0) on the same operands: bitwise, for SUM and MEAN
aggregation, empty receivers, a partial last tile and the optional stored aggregate
(mgnLayer.py NodeBlock and :144-146's scatter). Model-level parity against the oracle runs through
it in tests/test_gpu_parity.py (inference layers)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"
H = 128


class NodeChain:
    def __init__(self, seed, nlin=4):
        from aerognn.core import Pack
        from aerognn.functions import ChainSpec
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.nlin = nlin
        self.w = [(torch.randn(H, 2 * H, generator=g) * (2 * H) ** -0.5).to(DEV)] + \
                 [(torch.randn(H, H, generator=g) * H ** -0.5).to(DEV) for _ in range(nlin - 1)]
        self.b = [(torch.randn(H, generator=g) * 0.1).to(DEV) for _ in range(nlin)]
        self.gamma = (1.0 + 0.1 * torch.randn(H, generator=g)).to(DEV)
        self.beta = (0.1 * torch.randn(H, generator=g)).to(DEV)
        self.pack = Pack()
        self.spec = ChainSpec(list(zip(self.w, self.b)), (self.gamma, self.beta), H, self.pack, "n")
        self.pack.update(torch.bfloat16, torch.device(DEV))


def _graph(N, E, seed, empty_frac=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    dst = torch.randint(0, N, (E,), generator=g)
    if empty_frac:
        keep = torch.rand(N, generator=g) >= empty_frac
        dst = torch.nonzero(keep).flatten()[torch.randint(0, int(keep.sum()), (E,), generator=g)]
    dst = torch.sort(dst).values
    rowptr = torch.zeros(N + 1, dtype=torch.int64)
    rowptr[1:] = torch.cumsum(torch.bincount(dst, minlength=N), 0)
    return rowptr.to(torch.int32).to(DEV)


def _run(ch, x, ep, rowptr, kind, store, resident, saves=False):
    from aerognn import core
    from aerognn import _lib as L
    from aerognn.functions import _alloc_saves
    lib = L.lib()
    n0 = lib.agn_debug_node32_launches()
    old = lib.agn_set_option(L.OPT_RESIDENT, int(resident))
    try:
        out = torch.full_like(x, float("nan"))
        agg = torch.full_like(x, float("nan")) if store else None
        acts = hpre = stats = None
        if saves:  # the training saves as the model allocates them, zeroed (padding rows compare equal)
            acts, hpre, stats = _alloc_saves(ch.spec, x.shape[0], torch.bfloat16, x.device, True)
            for t in acts + [hpre, stats]:
                t.zero_()
            for t in acts:
                t.agn_mask.zero_()
        core.mlp_forward(rows=x.shape[0], dtype=torch.bfloat16, hidden=H, nlin=ch.nlin, out_dim=H,
                         segs=[(L.SEG_PLAIN, H, x.stride(0), x, None, None), (kind, H, ep.stride(0), ep, rowptr, agg)],
                         wpk=ch.spec.wpk(), bias=ch.spec.biases(), ln=ch.spec.lnp(), resid=x, out=out,
                         acts=acts, hpre=hpre, stats=stats)
        torch.cuda.synchronize()
    finally:
        lib.agn_set_option(L.OPT_RESIDENT, old)
    # the resident run went through node32_fwd_kernel, the other through the general kernel
    assert lib.agn_debug_node32_launches() - n0 == int(resident)
    sv = [] if not saves else [t for a in acts for t in (a, a.agn_mask)] + [hpre, stats]
    return out, agg, sv


@pytest.mark.parametrize("N,deg,kind,empty,store,nlin", [
    (70000, 6, "sum", 0.0, False, 4), (70001, 6, "mean", 0.0, True, 4), (65537, 3, "sum", 0.3, True, 4),
    (100000, 1, "mean", 0.5, False, 4), (66000, 40, "sum", 0.0, False, 4), (70000, 6, "sum", 0.0, False, 3),
    (65537, 3, "mean", 0.3, True, 3)])
def test_node32_bitwise_general(N, deg, kind, empty, store, nlin):
    from aerognn import _lib as L
    ch = NodeChain(31, nlin)
    E = N * deg
    rowptr = _graph(N, E, 32, empty)
    g = torch.Generator(device="cpu").manual_seed(33)
    x = torch.randn(N, H, generator=g).to(torch.bfloat16).to(DEV)
    ep = torch.randn(E, H, generator=g).to(torch.bfloat16).to(DEV)
    k = L.SEG_SUM if kind == "sum" else L.SEG_MEAN
    ref, ref_agg, _ = _run(ch, x, ep, rowptr, k, store, False)
    out, agg, _ = _run(ch, x, ep, rowptr, k, store, True)
    assert bool(torch.isfinite(ref.float()).all())
    assert torch.equal(out, ref)
    if store:
        assert torch.equal(agg, ref_agg)


@pytest.mark.parametrize("N,deg,nlin", [(70000, 6, 4), (65600, 2, 4), (70000, 6, 3)])
def test_node32_training_saves_bitwise_general(N, deg, nlin):
    """With the training saves (ReLU outputs and their mask bits, pre-LayerNorm rows, statistics,
    the aggregate) as the model allocates them."""
    from aerognn import _lib as L
    ch = NodeChain(34, nlin)
    E = N * deg
    rowptr = _graph(N, E, 35, 0.1)
    g = torch.Generator(device="cpu").manual_seed(36)
    x = torch.randn(N, H, generator=g).to(torch.bfloat16).to(DEV)
    ep = torch.randn(E, H, generator=g).to(torch.bfloat16).to(DEV)
    ref, ref_agg, ref_sv = _run(ch, x, ep, rowptr, L.SEG_SUM, True, False, saves=True)
    out, agg, sv = _run(ch, x, ep, rowptr, L.SEG_SUM, True, True, saves=True)
    assert torch.equal(out, ref) and torch.equal(agg, ref_agg)
    assert len(sv) == 2 * (nlin - 1) + 2
    for a, b in zip(sv, ref_sv):
        assert torch.equal(a, b)


@pytest.mark.parametrize("N,deg", [(70000, 6), (65601, 3)])
def test_node32_backward_bitwise_general(N, deg):
    """The resident node MLP backward (csrc/node32_bwd.hip, picked inside agn_mlp_backward) against
    the general kernel (AGN_OPT_RESIDENT = 0) on the forward's own saves: the pre-activation
    gradients G_3..G_0 (AGN_TILED), dx (+ the residual's g), dagg and the LayerNorm partial rows,
    bitwise; a partial last tile and a partial last 128-row block included."""
    from aerognn import core
    from aerognn import _lib as L
    from aerognn.functions import _alloc_gpre
    ch = NodeChain(51, 4)
    E = N * deg
    rowptr = _graph(N, E, 52, 0.1)
    g = torch.Generator(device="cpu").manual_seed(53)
    x = torch.randn(N, H, generator=g).to(torch.bfloat16).to(DEV)
    ep = torch.randn(E, H, generator=g).to(torch.bfloat16).to(DEV)
    gx = torch.randn(N, H, generator=g).to(torch.bfloat16).to(DEV)
    _, agg, sv = _run(ch, x, ep, rowptr, L.SEG_SUM, True, True, saves=True)
    acts = [sv[0], sv[2], sv[4]]
    hpre, stats = sv[6], sv[7]
    lib = L.lib()
    res = []
    for resident in (False, True):
        n0 = lib.agn_debug_node32_bwd_launches()
        old = lib.agn_set_option(L.OPT_RESIDENT, int(resident))
        try:
            gpre = _alloc_gpre(ch.spec, N, torch.bfloat16, x.device)
            for t in gpre:
                t.zero_()
            dx = torch.full_like(x, float("nan"))
            dagg = torch.full_like(x, float("nan"))
            part = torch.full((core.bwd_nblocks(N), 2 * H), float("nan"), dtype=torch.float32, device=DEV)
            nb = core.mlp_backward(rows=N, dtype=torch.bfloat16, hidden=H, nlin=4, out_dim=H, in_dim=2 * H,
                                   wtpk=ch.spec.wtpk(), acts=acts, g=gx, gpre=gpre, ln_g=ch.spec.lnp()[0],
                                   hpre=hpre, stats=stats, din=[(H, dx, True), (H, dagg, False)], ln_partial=part)
            torch.cuda.synchronize()
        finally:
            lib.agn_set_option(L.OPT_RESIDENT, old)
        assert lib.agn_debug_node32_bwd_launches() - n0 == int(resident)
        res.append((nb, gpre, dx, dagg, part))
    (nb0, gp0, dx0, da0, p0), (nb1, gp1, dx1, da1, p1) = res
    assert nb0 == nb1 == core.bwd_nblocks(N)
    assert bool(torch.isfinite(dx0.float()).all()) and bool(torch.isfinite(p0).all())
    assert torch.equal(dx1, dx0) and torch.equal(da1, da0)
    for a, b in zip(gp1, gp0):
        assert torch.equal(a, b)
    assert torch.equal(p1, p0)
