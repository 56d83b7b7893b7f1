"""The resident encoder MLP forward on narrow rows (csrc/enc32_fwd.hip), which agn_mlp_forward
picks for the node / edge encoders (k <= 16 input features, PLAIN or GATHER rows), against the
general kernel's narrow-input mode (AGN_OPT_RESIDENT = 0) on the same operands: bitwise, with and
without the training saves (mlp.py MLP, the encoders of models/bsms_mgn.py)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"
H = 128


class EncChain:
    def __init__(self, seed, k, nlin):
        from aerognn.core import Pack
        from aerognn.functions import ChainSpec
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.nlin = nlin
        self.w = [(torch.randn(H, k, generator=g) * k ** -0.5).to(DEV)] + \
                 [(torch.randn(H, H, generator=g) * H ** -0.5).to(DEV) for _ in range(nlin - 1)]
        self.b = [(torch.randn(H, generator=g) * 0.1).to(DEV) for _ in range(nlin)]
        self.gamma = (1.0 + 0.1 * torch.randn(H, generator=g)).to(DEV)
        self.beta = (0.1 * torch.randn(H, generator=g)).to(DEV)
        self.pack = Pack()
        self.spec = ChainSpec(list(zip(self.w, self.b)), (self.gamma, self.beta), H, self.pack, "x")
        self.pack.update(torch.bfloat16, torch.device(DEV))


def _run(ch, x, idx, resident, saves):
    from aerognn import core
    from aerognn import _lib as L
    from aerognn.functions import _alloc_saves
    lib = L.lib()
    n0 = lib.agn_debug_enc32_launches()
    old = lib.agn_set_option(L.OPT_RESIDENT, int(resident))
    rows = x.shape[0] if idx is None else idx.numel()
    try:
        out = torch.full((rows, H), float("nan"), dtype=torch.bfloat16, device=DEV)
        acts = hpre = stats = None
        if saves:
            acts, hpre, stats = _alloc_saves(ch.spec, rows, torch.bfloat16, x.device, True)
            for t in acts + [hpre, stats]:
                t.zero_()
            for t in acts:
                t.agn_mask.zero_()
        seg = (L.SEG_PLAIN, x.shape[1], x.stride(0), x, None, None) if idx is None else \
            (L.SEG_GATHER, x.shape[1], x.stride(0), x, idx, None)
        core.mlp_forward(rows=rows, dtype=torch.bfloat16, hidden=H, nlin=ch.nlin, out_dim=H, segs=[seg],
                         wpk=ch.spec.wpk(), bias=ch.spec.biases(), ln=ch.spec.lnp(), out=out,
                         acts=acts, hpre=hpre, stats=stats)
        torch.cuda.synchronize()
    finally:
        lib.agn_set_option(L.OPT_RESIDENT, old)
    assert lib.agn_debug_enc32_launches() - n0 == int(resident)
    sv = [] if not saves else [t for a in acts for t in (a, a.agn_mask)] + [hpre, stats]
    return out, sv


@pytest.mark.parametrize("rows,k,gather,nlin,saves", [
    (400001, 4, True, 3, False), (70000, 6, False, 3, False), (65537, 4, False, 4, False),
    (100000, 16, True, 3, True), (70001, 6, False, 3, True), (66000, 3, True, 4, True)])
def test_enc32_bitwise_general(rows, k, gather, nlin, saves):
    ch = EncChain(41, k, nlin)
    g = torch.Generator(device="cpu").manual_seed(42)
    n_in = rows + 123
    x = torch.randn(n_in, k, generator=g).to(torch.bfloat16).to(DEV)
    idx = torch.randperm(n_in, generator=g)[:rows].to(torch.int32).to(DEV) if gather else None
    if not gather:
        x = x[:rows]
    ref, ref_sv = _run(ch, x, idx, False, saves)
    out, sv = _run(ch, x, idx, True, saves)
    assert bool(torch.isfinite(ref.float()).all())
    assert torch.equal(out, ref)
    for a, b in zip(sv, ref_sv):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rows,out_dim,nlin,saves", [(70000, 3, 4, False), (65537, 4, 3, True), (100001, 32, 4, True)])
def test_dec32_bitwise_general(rows, out_dim, nlin, saves):
    """The resident decoder forward (dec32_fwd_kernel: H-wide rows to <= 32 outputs, no LayerNorm)
    against the general kernel's narrow-output mode, bitwise, with and without training saves (the
    saves variant runs 12 waves per CU)."""
    from aerognn import core
    from aerognn import _lib as L
    from aerognn.core import Pack
    from aerognn.functions import ChainSpec, _alloc_saves
    g = torch.Generator(device="cpu").manual_seed(61)
    ws = [(torch.randn(H, H, generator=g) * H ** -0.5).to(DEV) for _ in range(nlin - 1)] + \
         [(torch.randn(out_dim, H, generator=g) * H ** -0.5).to(DEV)]
    bs = [(torch.randn(H, generator=g) * 0.1).to(DEV) for _ in range(nlin - 1)] + \
         [(torch.randn(out_dim, generator=g) * 0.1).to(DEV)]
    pack = Pack()
    spec = ChainSpec(list(zip(ws, bs)), None, H, pack, "d")
    pack.update(torch.bfloat16, torch.device(DEV))
    x = torch.randn(rows, H, generator=g).to(torch.bfloat16).to(DEV)
    lib = L.lib()
    res = []
    for resident in (False, True):
        n0 = lib.agn_debug_dec32_launches()
        old = lib.agn_set_option(L.OPT_RESIDENT, int(resident))
        try:
            out = torch.full((rows, out_dim), float("nan"), dtype=torch.bfloat16, device=DEV)
            acts = None
            if saves:
                acts, _, _ = _alloc_saves(spec, rows, torch.bfloat16, x.device, True)
                for t in acts:
                    t.zero_()
                    t.agn_mask.zero_()
            core.mlp_forward(rows=rows, dtype=torch.bfloat16, hidden=H, nlin=nlin, out_dim=out_dim,
                             segs=[(L.SEG_PLAIN, H, x.stride(0), x, None, None)], wpk=spec.wpk(),
                             bias=spec.biases(), out=out, acts=acts)
            torch.cuda.synchronize()
        finally:
            lib.agn_set_option(L.OPT_RESIDENT, old)
        assert lib.agn_debug_dec32_launches() - n0 == int(resident)
        res.append((out, [] if acts is None else [t for a in acts for t in (a, a.agn_mask)]))
    (o0, s0), (o1, s1) = res
    assert bool(torch.isfinite(o0.float()).all())
    assert torch.equal(o1, o0)
    for a, b in zip(s1, s0):
        assert torch.equal(a, b)


@pytest.mark.parametrize("rows,out_dim,nlin,rowmajor", [(70000, 3, 4, ()), (65537, 4, 3, (0,)), (100001, 32, 4, (1,))])
def test_dec32_backward_bitwise_general(rows, out_dim, nlin, rowmajor):
    """The resident decoder backward (csrc/node32_bwd.hip dec32_bwd_kernel, picked inside
    agn_mlp_backward) against the general kernel's narrow-output mode (AGN_OPT_RESIDENT = 0) on the
    forward's own saves: every pre-activation gradient (tiled and row-major) and dx, bitwise; a
    partial last tile included."""
    from aerognn import core
    from aerognn import _lib as L
    from aerognn.core import Pack
    from aerognn.functions import ChainSpec, _alloc_saves, _alloc_gpre
    g = torch.Generator(device="cpu").manual_seed(71)
    ws = [(torch.randn(H, H, generator=g) * H ** -0.5).to(DEV) for _ in range(nlin - 1)] + \
         [(torch.randn(out_dim, H, generator=g) * H ** -0.5).to(DEV)]
    bs = [(torch.randn(H, generator=g) * 0.1).to(DEV) for _ in range(nlin - 1)] + \
         [(torch.randn(out_dim, generator=g) * 0.1).to(DEV)]
    pack = Pack()
    spec = ChainSpec(list(zip(ws, bs)), None, H, pack, "d")
    pack.update(torch.bfloat16, torch.device(DEV))
    x = torch.randn(rows, H, generator=g).to(torch.bfloat16).to(DEV)
    gy = torch.randn(rows, out_dim, generator=g).to(torch.bfloat16).to(DEV)
    out = torch.empty(rows, out_dim, dtype=torch.bfloat16, device=DEV)
    acts, _, _ = _alloc_saves(spec, rows, torch.bfloat16, x.device, True)
    core.mlp_forward(rows=rows, dtype=torch.bfloat16, hidden=H, nlin=nlin, out_dim=out_dim,
                     segs=[(L.SEG_PLAIN, H, x.stride(0), x, None, None)], wpk=spec.wpk(),
                     bias=spec.biases(), out=out, acts=acts)
    lib = L.lib()
    res = []
    for resident in (False, True):
        n0 = lib.agn_debug_dec32_bwd_launches()
        old = lib.agn_set_option(L.OPT_RESIDENT, int(resident))
        try:
            gpre = _alloc_gpre(spec, rows, torch.bfloat16, x.device, rowmajor)
            for t in gpre:
                t.zero_()
            dx = torch.full_like(x, float("nan"))
            nb = core.mlp_backward(rows=rows, dtype=torch.bfloat16, hidden=H, nlin=nlin, out_dim=out_dim,
                                   in_dim=H, wtpk=spec.wtpk(), acts=acts, g=gy, gpre=gpre,
                                   din=[(H, dx, False)])
            torch.cuda.synchronize()
        finally:
            lib.agn_set_option(L.OPT_RESIDENT, old)
        assert lib.agn_debug_dec32_bwd_launches() - n0 == int(resident)
        res.append((nb, gpre, dx))
    (nb0, gp0, dx0), (nb1, gp1, dx1) = res
    assert nb0 == nb1
    assert bool(torch.isfinite(dx0.float()).all())
    assert torch.equal(dx1, dx0)
    for a, b in zip(gp1, gp0):
        assert torch.equal(a, b)
