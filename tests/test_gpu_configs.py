"""GPU parity at every BASELINE.json configuration, the reference's bf16 mode, and the edge cases
of the drop-in boundary.

* C2 (MGN-15, 100k nodes / 598,400 edges, fp32): the whole model forward vs the CPU oracle at the
  fp32 bar (rel-L2 and max-element <= 1e-5).
* C4 (BSMS-4 over PyG-collated micro-batches of ellipsoid(400,250) meshes): the pooling maps of
  one full 8-mesh micro-batch bit-exact at all three levels, and the fp32 forward of a 2-mesh
  batch vs the oracle at 1e-5.
* C5 (5M nodes / 29,990,000 edges, 6 levels, bf16): all five pooling levels bit-exact vs the
  oracle, and the full-size bf16 forward deterministic and finite.
* bf16: the whole C3 architecture in bf16 vs the fp32 oracle (reported; SURVEY §8 does not gate
  it), and the reference's own bf16 mode (`model.to(torch.bfloat16)`: bf16 parameters) vs the
  reference's bf16 outputs in tests/golden/layer_bf16.npz.
* fp16: the reference's fp16 mode (fp16 parameters) vs its own fp16 outputs
  (tests/golden/layer_fp16_h{32,128}.npz), and fp16 activations through a BSMS model.
* edge cases: empty U-Net blocks (layers_per_scale=0 / [0, 2]), mixed +0.0/-0.0 and NaN x in the
  pooling sort, grouped-but-unsorted and gapped `batch` ids (unique_consecutive semantics,
  bsms_mgn.py:231-238), the hierarchy cache on reordered same-topology meshes, and guard bytes
  after every ReLU-mask / saved-activation buffer.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import load, max_rel, params, rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"
FWD = 1e-5
# 3x the measured full-size bf16-vs-fp32 rel-L2, 8.92e-3 (profiles/r3_gpu_evidence_tests.log)
C3_BF16_GATE = 2.7e-2


def _mesh(nu, nv, seed=0):
    from aerognn.meshgen import ellipsoid
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=seed).items()}


def _batch(nu, nv, seeds):
    from aerognn.meshgen import collate, ellipsoid
    return {k: torch.from_numpy(v) for k, v in collate([ellipsoid(nu, nv, seed=s) for s in seeds]).items()}


def _kw(S=4, P=15, H=128, lps=2):
    return dict(processor_size=P, num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
                hidden_dim_processor=H, hidden_dim_node_encoder=H, hidden_dim_edge_encoder=H, hidden_dim_decoder=H,
                aggregation="add", do_concat_trick=True, num_scales=S, layers_per_scale=lps, stride=2)


def _gate(got, ref, tol=FWD, what=""):
    got = got.detach().float().cpu()
    r, m = rel_l2(got, ref), max_rel(got, ref)
    print(f"{what}: rel-L2 {r:.2e}, max-elem {m:.2e}")
    assert r <= tol and m <= tol, (what, r, m)


def _eq(a, b):
    """Bitwise-equal values, NaN == NaN (a NaN coordinate propagates into pooled positions)."""
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.is_floating_point():
        return bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())
    return torch.equal(a, b)


def _maps_equal(got, ref, what):
    cn, ce, cei, cb, cp, f2c = [t.cpu() for t in got]
    assert torch.equal(f2c, ref[5]), what
    assert torch.equal(cei, ref[2]), what
    assert torch.equal(cb, ref[3]), what
    assert _eq(cn, ref[0]) and _eq(ce, ref[1]), what
    if ref[4] is not None:
        assert _eq(cp, ref[4]), what


def _levels_vs_oracle(t, nlev, width=8):
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    N, E = t["x"].shape[0], t["edge_index"].shape[1]
    g = torch.Generator().manual_seed(7)
    node = torch.randn(N, width, generator=g)
    edge = torch.randn(E, width, generator=g)
    batch = t.get("batch", torch.zeros(N, dtype=torch.long))
    model = BiStridedMeshGraphNet(6, 4, 4, hidden_dim_processor=width, stride=2).to(DEV)
    ref = (node, edge, t["edge_index"], batch, t["pos"])
    got = tuple(v.to(DEV) for v in ref)
    for lev in range(nlev):
        ref = R.downsample(*ref[:5], 2, stable=True)
        got = model._downsample(*got[:5])
        _maps_equal(got, ref, f"level {lev + 1}")
        print(f"level {lev + 1}: {ref[2].shape[1]} coarse edges, {ref[0].shape[0]} coarse nodes bit-exact")


# ------------------------------------------------------------------------------ C2
def test_c2_mgn15_fp32_forward_vs_oracle():
    from models.mgn import MeshGraphNet
    from oracle import refcpu as R
    t = _mesh(400, 250)
    assert (t["x"].shape[0], t["edge_index"].shape[1]) == (100000, 598400)
    kw = _kw()
    for k in ("num_scales", "layers_per_scale", "stride"):
        kw.pop(k)
    torch.manual_seed(0)
    model = MeshGraphNet(6, 4, 4, **kw).to(DEV)
    with torch.no_grad():
        pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV))
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = R.mgn_forward(p, t["x"], t["edge_attr"], t["edge_index"], R.cfg_from_kwargs(**kw))
    _gate(pred, ref, what="C2 MGN-15 fp32 forward")


# ------------------------------------------------------------------------------ C4
def test_c4_microbatch_pooling_maps_bitexact():
    t = _batch(400, 250, range(8))  # one micro-batch: 8 meshes, 800,000 nodes / 4,787,200 edges
    assert t["x"].shape[0] == 800000
    _levels_vs_oracle(t, 3)


def test_c4_two_meshes_fp32_forward_vs_oracle():
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    t = _batch(400, 250, (0, 1))
    kw = _kw()
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    with torch.no_grad():
        pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV), batch=t["batch"].to(DEV),
                     pos=t["pos"].to(DEV))
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], R.cfg_from_kwargs(**kw), t["batch"],
                             t["pos"], stable=True)
    _gate(pred, ref, what="C4 2-mesh BSMS-4 fp32 forward")


# ------------------------------------------------------------------------------ C5
def test_c5_pooling_maps_all_five_levels_bitexact():
    t = _mesh(2500, 2000)
    assert (t["x"].shape[0], t["edge_index"].shape[1]) == (5000000, 29990000)
    _levels_vs_oracle(t, 5, width=1)  # the 6-level hierarchy: every one of its 5 poolings


def test_c5_bf16_forward_deterministic_finite():
    from models.bsms_mgn import BiStridedMeshGraphNet
    t = {k: v.to(DEV) for k, v in _mesh(2500, 2000).items()}
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **_kw(S=6)).to(DEV)
    x, ea = t["x"].bfloat16(), t["edge_attr"].bfloat16()
    outs = []
    with torch.no_grad():
        for _ in range(2):
            outs.append(model(x, ea, t["edge_index"], pos=t["pos"]).clone())
    torch.cuda.synchronize()
    assert outs[0].shape == (5000000, 4)
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------------------------ bf16
def test_c3_architecture_bf16_vs_fp32_oracle_reported():
    """Whole-model bf16 error (bf16 activations, fp32 master weights) of the C3 architecture
    against the fp32 oracle on an oracle-sized mesh. SURVEY §8: reported, not gated; the assert
    is only a sanity bound."""
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    t = _mesh(100, 60)
    kw = _kw()
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    args = (t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV))
    with torch.no_grad():
        p32 = model(*args, pos=t["pos"].to(DEV))
        pbf = model(args[0].bfloat16(), args[1].bfloat16(), args[2], pos=t["pos"].to(DEV))
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], R.cfg_from_kwargs(**kw), None, t["pos"],
                             stable=True)
    r32, rbf = rel_l2(p32.float().cpu(), ref), rel_l2(pbf.float().cpu(), ref)
    print(f"BSMS-4 (15 layers, H=128) on 6,000 nodes: fp32 rel-L2 {r32:.2e}, bf16 rel-L2 {rbf:.2e} vs fp32 oracle")
    assert r32 <= FWD
    # 3x the measured 8.84e-3 (profiles/r2_gpu_tests_verbose.log): a regression gate, not a spec
    assert np.isfinite(rbf) and rbf <= 2.7e-2


def test_c3_full_size_bf16_vs_fp32_hip():
    """Whole-model bf16 error at the headline size (1M nodes / 5,996,000 edges, BSMS-4, 15
    layers): bf16 activations against the fp32 HIP path on the same model and mesh. The fp32 path
    is oracle-pinned at the 1e-5 bar at C2 and C4 sizes (tests above); here it is the reference
    for the bf16 error the headline metric is measured at."""
    from models.bsms_mgn import BiStridedMeshGraphNet
    t = {k: v.to(DEV) for k, v in _mesh(1000, 1000).items()}
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **_kw()).to(DEV)
    with torch.no_grad():
        p32 = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).double()
        pbf = model(t["x"].bfloat16(), t["edge_attr"].bfloat16(), t["edge_index"], pos=t["pos"]).double()
    r = float((pbf - p32).norm() / p32.norm())
    mx = float((pbf - p32).abs().max() / p32.abs().max())
    print(f"C3 full size BSMS-4: bf16 vs fp32 HIP rel-L2 {r:.2e}, max-elem {mx:.2e}")
    assert np.isfinite(r) and r <= C3_BF16_GATE


def test_reference_bf16_mode_layer():
    """The reference's bf16 mode casts the module (`.to(torch.bfloat16)`, train.py:20-40): bf16
    parameters and activations. Compared with the reference's own bf16 outputs (golden) and with
    its fp32 outputs, at the bf16 bar (rel-L2 <= 2e-2)."""
    from models.mgnLayer import MeshGraphNetLayer
    d, m = load("layer_bf16")
    H = m["H"]
    layer = MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True)
    layer.load_state_dict(params(d))
    layer = layer.to(DEV).to(torch.bfloat16)
    x = d["x"].to(DEV).bfloat16().requires_grad_(True)
    e = d["e"].to(DEV).bfloat16().requires_grad_(True)
    xo, eo = layer(x, e, d["edge_index"].to(DEV))
    assert xo.dtype == torch.bfloat16 and eo.dtype == torch.bfloat16
    for got, key in ((xo, "x_out_bf16"), (eo, "e_out_bf16"), (xo, "x_out"), (eo, "e_out")):
        r = rel_l2(got.float().cpu(), d[key])
        print(f"bf16-parameter layer vs {key}: rel-L2 {r:.2e}")
        assert r <= 2e-2, (key, r)
    (xo.float().square().sum() + eo.float().square().sum()).backward()
    for n, prm in layer.named_parameters():
        assert prm.grad is not None and prm.grad.dtype == torch.bfloat16, n
        assert torch.isfinite(prm.grad.float()).all(), n


# ------------------------------------------------------------------------------ fp16
@pytest.mark.parametrize("H", [32, 128])
def test_reference_fp16_mode_layer(H):
    """The reference's fp16 mode (train.py:35-38: fp16 default dtype, fp16 parameters) against
    its own fp16 outputs (tests/golden/layer_fp16_h*.npz) and its fp32 outputs. fp16 keeps 11
    significant bits, so the bar is rel-L2 <= 5e-3; the backward runs and gives finite fp16
    gradients."""
    from models.mgnLayer import MeshGraphNetLayer
    d, m = load(f"layer_fp16_h{H}")
    layer = MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True)
    layer.load_state_dict(params(d))
    layer = layer.to(DEV).to(torch.float16)
    x = d["x"].to(DEV).half().requires_grad_(True)
    e = d["e"].to(DEV).half().requires_grad_(True)
    xo, eo = layer(x, e, d["edge_index"].to(DEV))
    assert xo.dtype == torch.float16 and eo.dtype == torch.float16
    for got, key in ((xo, "x_out_fp16"), (eo, "e_out_fp16"), (xo, "x_out"), (eo, "e_out")):
        r = rel_l2(got.float().cpu(), d[key])
        print(f"fp16-parameter layer H={H} vs {key}: rel-L2 {r:.2e}")
        assert r <= 5e-3, (key, r)
    (xo.float().square().sum() + eo.float().square().sum()).backward()
    for n, prm in layer.named_parameters():
        assert prm.grad is not None and prm.grad.dtype == torch.float16, n
        assert torch.isfinite(prm.grad.float()).all(), n
    assert torch.isfinite(x.grad.float()).all() and torch.isfinite(e.grad.float()).all()


def test_bsms_fp16_activations_vs_fp32_oracle():
    """fp16 activations with fp32 master weights through the whole BSMS-4 model (general
    kernels; the resident kernels are bf16-only): forward vs the fp32 oracle, deterministic, and
    a full backward with finite gradients."""
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    t = _mesh(60, 40)
    kw = _kw(S=3, P=6, H=128)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    args = (t["x"].to(DEV).half(), t["edge_attr"].to(DEV).half(), t["edge_index"].to(DEV))
    with torch.no_grad():
        p1 = model(*args, pos=t["pos"].to(DEV))
        p2 = model(*args, pos=t["pos"].to(DEV))
    assert p1.dtype == torch.float16 and torch.equal(p1, p2)
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], R.cfg_from_kwargs(**kw), None, t["pos"],
                             stable=True)
    r = rel_l2(p1.float().cpu(), ref)
    print(f"BSMS-3 (6 layers, H=128) fp16 activations vs fp32 oracle: rel-L2 {r:.2e}")
    assert r <= 1e-2
    out = model(*args, pos=t["pos"].to(DEV))
    torch.nn.functional.mse_loss(out.float(), t["y"].to(DEV)).backward()
    for n, prm in model.named_parameters():
        assert prm.grad is not None and torch.isfinite(prm.grad).all(), n


# ------------------------------------------------------------------------------ edge cases
@pytest.mark.parametrize("lps", [0, [0, 2], [2, 0]])
def test_empty_unet_blocks_train(lps):
    """layers_per_scale = 0 or a list holding 0 (accepted by the reference's constructor,
    bsms_mgn.py:60-81): forward vs oracle and a full backward (an empty up block left
    an armed skip-gradient box)."""
    from aerognn.meshgen import ellipsoid, collate
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    t = {k: torch.from_numpy(v) for k, v in collate([ellipsoid(14, 9, seed=0), ellipsoid(10, 7, seed=1)]).items()}
    kw = _kw(S=3, P=5, H=32, lps=lps)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV), batch=t["batch"].to(DEV),
                 pos=t["pos"].to(DEV))
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    ref = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], R.cfg_from_kwargs(**kw), t["batch"], t["pos"],
                         stable=True)
    _gate(pred, ref.detach(), what=f"lps={lps}")
    torch.nn.functional.mse_loss(pred, t["y"].to(DEV)).backward()
    for n, prm in model.named_parameters():
        assert prm.grad is not None and torch.isfinite(prm.grad).all(), n


@pytest.mark.parametrize("case", ["isolated", "edgeless"])
def test_mgn_isolated_nodes_and_edgeless_graph(case):
    """Receivers with no incoming edges aggregate to 0 (torch_scatter's zero-initialised output),
    and a graph with no edges at all runs through the encoders, 5 layers and the decoder: forward
    vs the fp32 oracle at 1e-5, and a backward with finite gradients."""
    from models.mgn import MeshGraphNet
    from oracle import refcpu as R
    t = _mesh(20, 12)
    ei = t["edge_index"]
    if case == "isolated":
        keep = (ei[1] % 7 != 3) & (ei[0] % 11 != 5)  # every 7th node receives nothing, every 11th sends nothing
        ei = ei[:, keep].contiguous()
    else:
        ei = ei[:, :0].contiguous()
    ea = t["edge_attr"][: ei.shape[1]].contiguous()
    kw = _kw(P=5, H=32)
    for k in ("num_scales", "layers_per_scale", "stride"):
        kw.pop(k)
    torch.manual_seed(0)
    model = MeshGraphNet(6, 4, 4, **kw).to(DEV)
    pred = model(t["x"].to(DEV), ea.to(DEV), ei.to(DEV))
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = R.mgn_forward(p, t["x"], ea, ei, R.cfg_from_kwargs(**kw))
    _gate(pred, ref, what=f"MGN-5 {case}")
    torch.nn.functional.mse_loss(pred, t["y"].to(DEV)).backward()
    for n, prm in model.named_parameters():
        assert prm.grad is not None and torch.isfinite(prm.grad).all(), n


def test_bsms_batch_with_tiny_meshes():
    """Meshes of 6 and 12 nodes beside a normal one in one batch, 4 levels: the tiny graphs pool
    down to a single node (and no edges) before the bottom; forward vs the oracle at 1e-5 and a
    full backward."""
    from aerognn.meshgen import collate, ellipsoid
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    t = {k: torch.from_numpy(v) for k, v in collate([ellipsoid(3, 2, seed=0), ellipsoid(16, 10, seed=1),
                                                      ellipsoid(4, 3, seed=2)]).items()}
    kw = _kw(S=4, P=7, H=32)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV), batch=t["batch"].to(DEV),
                 pos=t["pos"].to(DEV))
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    with torch.no_grad():
        ref = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], R.cfg_from_kwargs(**kw), t["batch"],
                             t["pos"], stable=True)
    _gate(pred, ref, what="BSMS-4 tiny meshes")
    torch.nn.functional.mse_loss(pred, t["y"].to(DEV)).backward()
    for n, prm in model.named_parameters():
        assert prm.grad is not None and torch.isfinite(prm.grad).all(), n


def test_signed_zero_and_nan_x_pool_like_torch_argsort():
    """-0.0 and +0.0 compare equal in torch.argsort (stable tie rule: node id decides) and NaN
    sorts last: the pooling keys follow."""
    t = _batch(16, 10, (0, 1))
    pos = t["pos"].clone()
    n = pos.shape[0]
    sel = torch.arange(0, n, 7)
    pos[sel, 0] = torch.where(sel % 2 == 0, torch.tensor(0.0), torch.tensor(-0.0))
    pos[torch.arange(3, n, 41), 0] = float("nan")
    t["pos"] = pos
    _levels_vs_oracle(t, 2, width=4)


def test_unsorted_and_gapped_batch_ids():
    """Graph ids in grouped but unsorted order ([2.., 0.., 1..]) and with gaps ([1.., 3..]): the
    pooling visits graphs in unique_consecutive order and keeps the ids (bsms_mgn.py:231-256)."""
    from aerognn.meshgen import collate, ellipsoid
    ms = [ellipsoid(12, 8, seed=s) for s in range(3)]
    for ids in ([2, 0, 1], [1, 3, 4]):
        b = collate(ms)
        t = {k: torch.from_numpy(v) for k, v in b.items()}
        t["batch"] = torch.cat([torch.full((m["x"].shape[0],), g, dtype=torch.long) for g, m in zip(ids, ms)])
        _levels_vs_oracle(t, 2, width=4)


def test_hierarchy_cache_reordered_same_topology():
    """Two same-topology meshes swapped inside a micro-batch (C4's case) must not hit the other
    order's cache entry (What's weak 6)."""
    from aerognn.meshgen import collate, ellipsoid
    from models.bsms_mgn import BiStridedMeshGraphNet
    a, b = ellipsoid(20, 12, seed=0), ellipsoid(20, 12, seed=1)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **_kw(S=3, P=5, H=32)).to(DEV)

    def run(ms):
        t = {k: torch.from_numpy(v).to(DEV) for k, v in collate(ms).items()}
        with torch.no_grad():
            return model(t["x"], t["edge_attr"], t["edge_index"], batch=t["batch"], pos=t["pos"]).clone()
    ref_ab, ref_ba = run([a, b]), run([b, a])
    model.cache_hierarchy(True)
    for _ in range(2):
        assert torch.equal(run([a, b]), ref_ab)
        assert torch.equal(run([b, a]), ref_ba)
    assert len(model._hcache) == 2


def test_guard_bytes_after_saved_buffers(monkeypatch):
    """Every ReLU-mask and saved-activation buffer of a training forward gets 4 KB of sentinel
    bytes after its end; the resident and the general kernels must leave them untouched (the
    out-of-range mask store fixed in ea93d27 would fail this)."""
    import aerognn.functions as F
    from aerognn import core
    from models.mlp import MLP
    guards = []

    def guarded(t):
        flat = t.view(-1).view(torch.uint8)
        buf = torch.full((flat.numel() + 4096,), 0xA5, dtype=torch.uint8, device=t.device)
        out = buf[:flat.numel()].view(t.dtype).view(t.shape)
        for k in ("agn_tiled", "agn_rows"):
            if hasattr(t, k):
                setattr(out, k, getattr(t, k))
        guards.append(buf)
        return out

    real_mask, real_tiled = core.relu_mask_empty, core.tiled_empty
    monkeypatch.setattr(F, "relu_mask_empty", lambda *a, **k: guarded(real_mask(*a, **k)))
    monkeypatch.setattr(F, "tiled_empty", lambda *a, **k: guarded(real_tiled(*a, **k)))
    H = 128
    for rows in (100_003, 3_001):  # resident / general forward, ragged last tile
        for dtype in (torch.bfloat16, torch.float32):
            g = torch.Generator().manual_seed(5)
            x = torch.randn(rows, H, generator=g).to(DEV, dtype).requires_grad_(True)
            torch.manual_seed(0)
            mlp = MLP(H, H, H, num_hidden_layers=2).to(DEV)
            mlp(x).float().square().sum().backward()
    torch.cuda.synchronize()
    assert guards
    for buf in guards:
        assert bool((buf[-4096:] == 0xA5).all())
