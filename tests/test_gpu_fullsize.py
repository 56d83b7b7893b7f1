"""GPU parity at BASELINE.json sizes and on the large-row kernels.

* the persistent resident-weight edge kernels (used only for bf16 H=128 edge MLPs with
  >= 65,536 rows) are bitwise identical to the general kernels (agn_set_option A/B) for every
  activation and input gradient; parameter gradients agree to fp32 rounding (LayerNorm
  parameter partials are grouped per persistent block instead of per 128-row block);
* C2 size (100k nodes / 598,400 edges): one fp32 MeshGraphNetLayer vs the CPU oracle at the
  1e-5 bar;
* C3 size (1M nodes / 5,996,000 edges): the bi-stride pooling maps of the first two levels are
  bit-exact vs the oracle's `_downsample` (restated reference, bsms_mgn.py:217-301), and the
  full bf16 BSMS-4 train step is deterministic and finite (size-independent properties).
"""
import os

import numpy as np
import pytest
import torch

from golden_util import rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"


def _mesh(nu, nv, seed=0):
    from aerognn.meshgen import ellipsoid
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=seed).items()}


def _set_resident(v):
    from aerognn import _lib as L
    return L.lib().agn_set_option(L.OPT_RESIDENT, int(v))


def _layer_step(layer, x, e, lv):
    xg = x.clone().requires_grad_(True)
    eg = e.clone().requires_grad_(True)
    layer.zero_grad()
    xo, eo = layer.forward_level(xg, eg, lv)
    (xo.float().square().sum() + 0.5 * eo.float().square().sum()).backward()
    torch.cuda.synchronize()
    return xo.detach(), eo.detach(), xg.grad, eg.grad, {n: p.grad.clone() for n, p in layer.named_parameters()}


def test_resident_kernels_bitwise_equal_general():
    from aerognn.graph import Level
    from models.mgnLayer import MeshGraphNetLayer
    m = _mesh(150, 110)  # 16,500 nodes / 98,400 edges (> 65,536: resident path eligible)
    ei = m["edge_index"].to(DEV)
    N, E = m["x"].shape[0], ei.shape[1]
    assert E >= 65536
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).to(DEV)
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(N, 128, generator=g).to(DEV, torch.bfloat16)
    e = torch.randn(E, 128, generator=g).to(DEV, torch.bfloat16)
    old = _set_resident(1)
    try:
        res = _layer_step(layer, x, e, lv)
        _set_resident(0)
        gen = _layer_step(layer, x, e, lv)
    finally:
        _set_resident(old)
    for name, a, b in zip(("x'", "e'", "dx", "de"), res[:4], gen[:4]):
        r = rel_l2(a.float(), b.double())
        frac = float((a != b).float().mean())
        print(f"{name}: rel-L2 {r:.2e}, differing elements {frac:.2e}")
        assert torch.equal(a, b), (name, r, frac)
    worst = max(rel_l2(res[4][n].float(), gen[4][n].double()) for n in res[4])
    print(f"param grads worst rel-L2 {worst:.2e}")
    assert worst <= 1e-6


@pytest.mark.parametrize("nu,nv", [(150, 110), (97, 61)])  # 16,500 nodes; 5,917 nodes (ragged tile)
def test_proj_kernels_bitwise_equal_general(nu, nv, monkeypatch):
    """agn_proj_forward / agn_proj_backward (csrc/proj.hip, the node-row projections of the
    sum-trick edge block) against the general MLP kernel they replace (AEROGNN_PROJ_KERNEL=0):
    every output and gradient of a bf16 layer training step bitwise equal."""
    from aerognn.graph import Level
    from models.mgnLayer import MeshGraphNetLayer
    m = _mesh(nu, nv)
    ei = m["edge_index"].to(DEV)
    N, E = m["x"].shape[0], ei.shape[1]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).to(DEV)
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(2)
    x = torch.randn(N, 128, generator=g).to(DEV, torch.bfloat16)
    e = torch.randn(E, 128, generator=g).to(DEV, torch.bfloat16)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("AEROGNN_PROJ_KERNEL", flag)
        runs.append(_layer_step(layer, x, e, lv))
    a, b = runs
    for name, u, v in zip(("x'", "e'", "dx", "de"), a[:4], b[:4]):
        assert torch.equal(u, v), name
    for n in a[4]:
        assert torch.equal(a[4][n], b[4][n]), n


def test_resident_encoder_backward_bitwise_equal_general():
    """The edge encoder (MLP 4 -> 128, n_hid=2, LN; no input gradient) takes the resident
    backward too: gpre / parameter grads match the general kernel."""
    from models.mlp import MLP
    E = 100_000
    g = torch.Generator(device="cpu").manual_seed(3)
    ea = torch.randn(E, 4, generator=g).to(DEV, torch.bfloat16)
    gy = torch.randn(E, 128, generator=g).to(DEV, torch.bfloat16)
    torch.manual_seed(0)
    enc = MLP(4, 128, 128, num_hidden_layers=2).to(DEV)
    outs = []
    old = _set_resident(1)
    try:
        for flag in (1, 0):
            _set_resident(flag)
            enc.zero_grad()
            y = enc(ea)
            y.backward(gy)
            torch.cuda.synchronize()
            outs.append((y.detach(), {n: p.grad.clone() for n, p in enc.named_parameters()}))
    finally:
        _set_resident(old)
    assert torch.equal(outs[0][0], outs[1][0])
    worst = max(rel_l2(outs[0][1][n].float(), outs[1][1][n].double()) for n in outs[0][1])
    print(f"encoder param grads worst rel-L2 {worst:.2e}")
    assert worst <= 1e-6


def test_c2_layer_fp32_vs_oracle():
    from aerognn.graph import Level
    from models.mgnLayer import MeshGraphNetLayer
    from oracle import refcpu as R
    m = _mesh(400, 250)  # C2: 100,000 nodes / 598,400 edges
    N, E = m["x"].shape[0], m["edge_index"].shape[1]
    assert (N, E) == (100000, 598400)
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True)
    g = torch.Generator(device="cpu").manual_seed(2)
    x = torch.randn(N, 128, generator=g)
    e = torch.randn(E, 128, generator=g)
    p = {f"L.{k}": v for k, v in layer.state_dict().items()}
    cfg = R.cfg_from_kwargs(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                            do_concat_trick=True, aggregation="add")
    with torch.no_grad():
        xr, er = R.gmp_layer(p, "L", x, e, m["edge_index"], cfg)
    layer = layer.to(DEV)
    ei = m["edge_index"].to(DEV)
    with torch.no_grad():
        xo, eo = layer(x.to(DEV), e.to(DEV), ei)
    for got, ref in ((xo, xr), (eo, er)):
        got = got.cpu()
        r, m = rel_l2(got, ref), float((got - ref).abs().max()) / float(ref.abs().max())
        print(f"C2 layer: rel-L2 {r:.2e}, max-elem {m:.2e}")
        assert r <= 1e-5 and m <= 1e-5


@pytest.mark.parametrize("trick", [False, True])
def test_c2_layer_fp32_fwd_bwd_vs_oracle(trick):
    """One fp32 MeshGraphNetLayer at C2 size, forward AND backward, against the CPU oracle's
    float64 autograd: every output, input gradient and parameter gradient at the 1e-5 bar
    (rel-L2; outputs and input gradients also max-element). trick=False is the concat edge MLP
    (mgnLayer.py:10-49): hand-written kernels only (gathered-operand agn_wgrad for W_0's x_src /
    x_dst blocks, agn_segment_sum2 for dx + scatter(d x_src) + scatter(d x_dst)). Inputs are
    conditioned away from ReLU kinks (tests/kinkfree.py: rows re-drawn, none dropped)."""
    from kinkfree import kink_free
    from models.mgnLayer import MeshGraphNetLayer
    from oracle import refcpu as R
    m = _mesh(400, 250)  # C2: 100,000 nodes / 598,400 edges
    N, E = m["x"].shape[0], m["edge_index"].shape[1]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=trick)
    g = torch.Generator(device="cpu").manual_seed(4)
    x = torch.randn(N, 128, generator=g)
    e = torch.randn(E, 128, generator=g)
    gxo = torch.randn(N, 128, generator=g)
    geo = torch.randn(E, 128, generator=g)
    p64 = {f"L.{k}": v.double() for k, v in layer.state_dict().items()}
    cfg = R.cfg_from_kwargs(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                            do_concat_trick=trick, aggregation="add")
    ei = m["edge_index"]
    n = kink_free(lambda xx, ee: R.gmp_layer(p64, "L", xx, ee, ei, cfg), x, e, g)
    print(f"kink-free inputs: {n} rows re-drawn of {N + E}")
    p = {k: v.clone().requires_grad_(True) for k, v in p64.items()}
    xr_in, er_in = x.double().requires_grad_(True), e.double().requires_grad_(True)
    xr, er = R.gmp_layer(p, "L", xr_in, er_in, ei, cfg)
    torch.autograd.backward([xr, er], [gxo.double(), geo.double()])
    layer = layer.to(DEV)
    xg, eg = x.to(DEV).requires_grad_(True), e.to(DEV).requires_grad_(True)
    xo, eo = layer(xg, eg, ei.to(DEV))
    torch.autograd.backward([xo, eo], [gxo.to(DEV), geo.to(DEV)])
    torch.cuda.synchronize()
    pairs = [("x'", xo, xr), ("e'", eo, er), ("dx", xg.grad, xr_in.grad), ("de", eg.grad, er_in.grad)]
    pairs += [(n, q.grad, p[f"L.{n}"].grad) for n, q in layer.named_parameters()]
    worst = ("", 0.0)
    for name, got, ref in pairs:
        got, ref = got.detach().cpu().double(), ref.detach()
        r = rel_l2(got, ref)
        mx = float((got - ref).abs().max()) / max(float(ref.abs().max()), 1e-30)
        if name in ("x'", "e'", "dx", "de"):
            print(f"C2 {'sum' if trick else 'concat'} layer {name}: rel-L2 {r:.2e}, max-elem {mx:.2e}")
            assert r <= 1e-5 and mx <= 1e-5, (name, r, mx)
        worst = max(worst, (name, r), key=lambda t: t[1])
    print(f"C2 {'sum' if trick else 'concat'} layer param grads worst rel-L2 {worst[1]:.2e} ({worst[0]})")
    assert worst[1] <= 1e-5, worst


def test_c3_pooling_maps_bitexact_vs_oracle():
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    m = _mesh(1000, 1000)  # C3: 1,000,000 nodes / 5,996,000 edges
    N, E = m["x"].shape[0], m["edge_index"].shape[1]
    assert (N, E) == (1000000, 5996000)
    node = torch.randn(N, 8)
    edge = torch.randn(E, 8)
    batch = torch.zeros(N, dtype=torch.long)
    ref1 = R.downsample(node, edge, m["edge_index"], batch, m["pos"], 2, stable=True)
    ref2 = R.downsample(ref1[0], ref1[1], ref1[2], ref1[3], ref1[4], 2, stable=True)
    ref3 = R.downsample(ref2[0], ref2[1], ref2[2], ref2[3], ref2[4], 2, stable=True)  # all 3 C3 levels
    model = BiStridedMeshGraphNet(6, 4, 4, hidden_dim_processor=8, stride=2).to(DEV)
    got1 = model._downsample(node.to(DEV), edge.to(DEV), m["edge_index"].to(DEV), batch.to(DEV),
                             m["pos"].to(DEV))
    got2 = model._downsample(*[t for t in got1[:5]])
    got3 = model._downsample(*[t for t in got2[:5]])
    for got, ref in ((got1, ref1), (got2, ref2), (got3, ref3)):
        cn, ce, cei, cb, cp, f2c = [t.cpu() for t in got]
        assert torch.equal(f2c, ref[5])
        assert torch.equal(cei, ref[2])
        assert torch.equal(cb, ref[3])
        assert torch.equal(cn, ref[0]) and torch.equal(ce, ref[1]) and torch.equal(cp, ref[4])


def test_c3_train_step_deterministic_and_finite():
    from models.bsms_mgn import BiStridedMeshGraphNet
    m = _mesh(1000, 1000)
    t = {k: v.to(DEV) for k, v in m.items()}
    x, ea = t["x"].to(torch.bfloat16), t["edge_attr"].to(torch.bfloat16)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, processor_size=15, num_hidden_layers_node_processor=2,
                                  num_hidden_layers_edge_processor=2, num_hidden_layers_node_encoder=2,
                                  num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
                                  do_concat_trick=True, num_scales=4, layers_per_scale=2, stride=2).to(DEV)
    outs = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        pred = model(x, ea, t["edge_index"], batch=None, pos=t["pos"])
        torch.nn.functional.mse_loss(pred.float(), t["y"]).backward()
        outs.append((pred.detach().clone(), [p.grad.clone() for p in model.parameters()]))
    assert torch.isfinite(outs[0][0].float()).all()
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert torch.isfinite(a).all() and torch.equal(a, b)



def _decode_tiled(t, rows, H):
    """AGN_TILED [rows_pad, H] -> row-major [rows, H] (aerognn.h layout): bf16 unit (i, h) of row c
    holds features 16i+4h+{0..3}, 16i+8+4h+{0..3}; fp32 unit (i, h) features 8i+4h+{0..3}."""
    if t.dtype == torch.bfloat16:
        U, per, iv = H // 16, 8, torch.int16  # 16-B units per lane (half row)
    else:
        U, per, iv = H // 8, 4, torch.int32
    u = t.view(iv).reshape(-1, U, 2, 32, per)  # [tile][i][h][c][per]
    out = torch.empty(u.shape[0], 32, H, dtype=iv, device=t.device)
    for i in range(U):
        for hh in range(2):
            v = u[:, i, hh]
            if per == 8:
                out[:, :, 16 * i + 4 * hh:16 * i + 4 * hh + 4] = v[:, :, :4]
                out[:, :, 16 * i + 8 + 4 * hh:16 * i + 8 + 4 * hh + 4] = v[:, :, 4:]
            else:
                out[:, :, 8 * i + 4 * hh:8 * i + 4 * hh + 4] = v
    return out.reshape(-1, H)[:rows].view(t.dtype)


@pytest.mark.parametrize("rows", [100_000, 3_000])  # resident / general forward
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_relu_mask_matches_saved_activations(rows, dtype):
    """AGN_RELU_MASK bits written by the forward == (saved activation > 0) for every hidden layer:
    the backward's ReLU select reads these bits instead of the activations."""
    from models.mlp import MLP
    H = 128
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(rows, H, generator=g).to(DEV, dtype)
    torch.manual_seed(0)
    mlp = MLP(H, H, H, num_hidden_layers=2).to(DEV)
    y = mlp(x.requires_grad_(True))
    ctx = y.grad_fn
    torch.cuda.synchronize()
    assert len(ctx.acts) == 3  # num_hidden_layers=2: Lin, 2 hidden Lin, out Lin -> 3 ReLU outputs
    for act in ctx.acts:
        if getattr(act, "agn_tiled", False):
            a = _decode_tiled(act, rows, H).float()
        else:
            a = act[:rows].float()
        pos = (a > 0).cpu().numpy()  # [rows, H]
        ntile = (rows + 31) // 32
        m = act.agn_mask.cpu().numpy().astype(np.uint32).reshape(ntile, 2, 64)  # [tile][d][lane]
        rho = np.arange(64)
        bits = (m[:, rho // 32, :] >> (rho % 32)[None, :, None]) & 1  # [tile][rho][lane]
        lane = np.arange(64)
        c, h = lane % 32, lane // 32
        f = 8 * (rho[:, None] // 4) + 4 * h[None, :] + rho[:, None] % 4  # [rho][lane]
        r = (np.arange(ntile)[:, None, None] * 32 + c[None, None, :]).repeat(64, 1)  # [tile][rho][lane]
        ok = r < rows
        expect = pos[np.minimum(r, rows - 1), np.broadcast_to(f, r.shape)]
        assert np.array_equal(bits.astype(bool)[ok], expect[ok])


@pytest.mark.parametrize("E", [98_400, 70_001])  # ragged last round / ragged last tile
def test_fused_edge_bwd_matches_split(E, monkeypatch):
    """agn_edge_bwd_fused (forward recompute + LayerNorm backward + chain rule + dW1..dW3 in one
    persistent launch; the forward saves nothing) against the split path (saved activations,
    agn_mlp_backward + agn_wgrad): outputs, dx and de bitwise equal (same operands and MFMA order
    per row), parameter gradients equal up to the fp32 order of the row sums."""
    from aerognn.graph import Level
    from models.mgnLayer import MeshGraphNetLayer
    m = _mesh(150, 110)
    ei = m["edge_index"][:, :E].to(DEV)
    N = m["x"].shape[0]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).to(DEV)
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(N, 128, generator=g).to(DEV, torch.bfloat16)
    e = torch.randn(E, 128, generator=g).to(DEV, torch.bfloat16)
    monkeypatch.setenv("AEROGNN_FUSED_EDGE_BWD", "1")
    fused = _layer_step(layer, x, e, lv)
    monkeypatch.setenv("AEROGNN_FUSED_EDGE_BWD", "0")
    split = _layer_step(layer, x, e, lv)
    for name, a, b in zip(("x'", "e'", "dx", "de"), fused[:4], split[:4]):
        r = rel_l2(a.float(), b.double())
        print(f"{name}: rel-L2 {r:.2e}, differing {float((a != b).float().mean()):.2e}")
        assert torch.equal(a, b), (name, r)
    worst = 0.0
    for n in fused[4]:
        r = rel_l2(fused[4][n].float(), split[4][n].double())
        worst = max(worst, r)
        print(f"{n:45s} rel-L2 {r:.2e}")
    assert worst <= 1e-5, worst


@pytest.mark.parametrize("aggregation,dtype,E", [("add", torch.bfloat16, 98_400), ("mean", torch.bfloat16, 98_400),
                                                 ("add", torch.bfloat16, 70_001), ("add", torch.float32, 98_400)])
def test_node_aggregation_walk_equals_segment_sum(aggregation, dtype, E):
    """The receiver aggregation of the node update (mgnLayer.py:144-146) as the node kernel walks it
    (its SUM / MEAN input segment over each receiver's CSC range, stored for the backward in
    training) is bitwise agn_segment_sum of e' (fp32 in edge order, one rounding: torch_scatter's
    order). E = 70,001 (a prefix of the CSC edges) leaves a ragged last tile and receivers without
    edges; fp32 runs the general kernels."""
    from aerognn import core
    from aerognn.graph import Level
    from models.mgnLayer import MeshGraphNetLayer
    m = _mesh(150, 110)
    ei = m["edge_index"][:, :E].to(DEV)
    N = m["x"].shape[0]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, aggregation=aggregation, do_concat_trick=True).to(DEV, dtype)
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(N, 128, generator=g).to(DEV, dtype).requires_grad_(True)
    e = torch.randn(E, 128, generator=g).to(DEV, dtype).requires_grad_(True)
    xo, eo = layer.forward_level(x, e, lv)
    agg = xo.grad_fn.saves[6]  # the node kernel's stored SUM / MEAN segment (GMPFn ctx.saves)
    ref = core.segment_sum(N, 128, lv.rowptr, None, eo.detach(), torch.empty_like(agg), mean=(aggregation == "mean"))
    torch.cuda.synchronize()
    empty = int((lv.rowptr[1:] == lv.rowptr[:-1]).sum())
    print(f"{N} receivers ({empty} without edges): differing {float((agg != ref).float().mean()):.2e}")
    assert torch.equal(agg, ref)
