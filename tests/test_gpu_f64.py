"""float64 mode (train.py:20-40 precision "double"): the MLP / GMP path on the agn_f64_* kernels
and the graph ops' float64 instantiations, against the float64 oracle (oracle/refcpu.py, the
reference's aten sequence) on the same weights and inputs. Both sides compute in fp64; only the
summation orders differ, so outputs and every gradient agree to ~1e-13 (gate 1e-10 rel-L2)."""
import os

import numpy as np
import pytest
import torch

from golden_util import rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"
TOL = 1e-10


def _mesh(nu, nv, seed=0):
    from aerognn.meshgen import ellipsoid
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=seed).items()}


def _check(name, got, ref, tol=TOL):
    r = rel_l2(got.detach().cpu().double(), ref.detach().double())
    print(f"f64 {name}: rel-L2 {r:.3e}")
    assert r <= tol, (name, r)


@pytest.mark.parametrize("n_hid,in_dim,out_dim,ln,act", [(2, 10, 64, True, "relu"), (0, 7, 4, False, "relu"),
                                                         (1, 128, 128, True, "relu"), (2, 10, 64, True, "gelu"),
                                                         (2, 10, 64, True, "silu"), (2, 10, 64, True, "tanh")])
def test_f64_mlp_vs_oracle(n_hid, in_dim, out_dim, ln, act):
    from models.mlp import MLP
    from oracle import refcpu as R
    torch.manual_seed(0)
    m = MLP(in_dim, 128, out_dim, num_hidden_layers=n_hid, activation_fn=act, use_layer_norm=ln).double()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(3001, in_dim, generator=g, dtype=torch.float64)
    gy = torch.randn(3001, out_dim, generator=g, dtype=torch.float64)
    p = {f"m.{k}": v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    xr = x.clone().requires_grad_(True)
    ref = R.mlp(p, "m", xr, R.mlp_nlin(n_hid), ln=ln, act=R.act_of({"activation_fn": act}))
    ref.backward(gy)
    m = m.to(DEV)
    xg = x.to(DEV).requires_grad_(True)
    y = m(xg)
    assert y.dtype == torch.float64
    y.backward(gy.to(DEV))
    _check("mlp out", y, ref)
    _check("mlp dx", xg.grad, xr.grad)
    for n, q in m.named_parameters():
        _check(f"mlp d{n}", q.grad, p[f"m.{n}"].grad)


@pytest.mark.parametrize("trick,aggregation", [(True, "add"), (False, "add"), (True, "mean"), (False, "mean")])
def test_f64_gmp_layer_fwd_bwd_vs_oracle(trick, aggregation):
    """MeshGraphNetLayer (mgnLayer.py:177-213) in fp64: sum trick and concat edge block, add and
    mean aggregation; x', e', dx, de and every parameter gradient."""
    from models.mgnLayer import MeshGraphNetLayer
    from oracle import refcpu as R
    m = _mesh(60, 50)
    ei = m["edge_index"]
    N, E = m["x"].shape[0], ei.shape[1]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, aggregation=aggregation, do_concat_trick=trick).double()
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, 128, generator=g, dtype=torch.float64)
    e = torch.randn(E, 128, generator=g, dtype=torch.float64)
    gx = torch.randn(N, 128, generator=g, dtype=torch.float64)
    ge = torch.randn(E, 128, generator=g, dtype=torch.float64)
    p = {f"L.{k}": v.detach().clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    cfg = R.cfg_from_kwargs(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                            do_concat_trick=trick, aggregation=aggregation)
    xr, er = x.clone().requires_grad_(True), e.clone().requires_grad_(True)
    xo_r, eo_r = R.gmp_layer(p, "L", xr, er, ei, cfg)
    torch.autograd.backward([xo_r, eo_r], [gx, ge])
    layer = layer.to(DEV)
    xg, eg = x.to(DEV).requires_grad_(True), e.to(DEV).requires_grad_(True)
    xo, eo = layer(xg, eg, ei.to(DEV))
    torch.autograd.backward([xo, eo], [gx.to(DEV), ge.to(DEV)])
    _check("x'", xo, xo_r)
    _check("e'", eo, eo_r)
    _check("dx", xg.grad, xr.grad)
    _check("de", eg.grad, er.grad)
    for n, q in layer.named_parameters():
        _check(f"d{n}", q.grad, p[f"L.{n}"].grad)


def test_f64_layer_gelu_golden():
    """The reference's float64 MeshGraphNetLayer with activation_fn='gelu' (tests/golden, made by
    tools/make_goldens.py from the reference itself): the node chain on GELU, the sum-trick edge
    chain on ReLU (mgnLayer.py:81)."""
    from golden_util import load, params
    from models.mgnLayer import MeshGraphNetLayer
    d, m = load("layer_sum_h32_f64_gelu")
    H, nh = m["H"], m["n_hid"]
    layer = MeshGraphNetLayer(H, H, H, nh, nh, "gelu", True, m["aggregation"], m["trick"]).double()
    layer.load_state_dict(params(d))
    layer = layer.to(DEV)
    x = d["x"].to(DEV).requires_grad_(True)
    e = d["e"].to(DEV).requires_grad_(True)
    xo, eo = layer(x, e, d["edge_index"].to(DEV))
    torch.autograd.backward([xo, eo], [d["gx_out"].to(DEV), d["ge_out"].to(DEV)])
    _check("x'", xo, d["x_out"])
    _check("e'", eo, d["e_out"])
    _check("dx", x.grad, d["gx"])
    _check("de", e.grad, d["ge"])
    for n, q in layer.named_parameters():
        _check(f"d{n}", q.grad, d["gp:" + n])


@pytest.mark.parametrize("kind", ["mgn", "bsms"])
def test_f64_model_train_step_vs_oracle(kind):
    """A whole MeshGraphNet-5 / BSMS-4 (15 layers) train step in fp64: prediction, loss and every
    parameter gradient against the float64 oracle (pooling maps from fp32 position keys, the
    same as the oracle's on these tie-free meshes)."""
    from oracle import refcpu as R
    t = _mesh(40, 30)
    kw = dict(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
              num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
              aggregation="add", do_concat_trick=True)
    torch.manual_seed(0)
    if kind == "mgn":
        from models.mgn import MeshGraphNet
        kw.update(processor_size=5)
        model = MeshGraphNet(6, 4, 4, **kw).double()
    else:
        from models.bsms_mgn import BiStridedMeshGraphNet
        kw.update(processor_size=15, num_scales=4, layers_per_scale=2, stride=2)
        model = BiStridedMeshGraphNet(6, 4, 4, **kw).double()
    x, ea, y = t["x"].double(), t["edge_attr"].double(), t["y"].double()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    cfg = R.cfg_from_kwargs(**kw)
    if kind == "mgn":
        ref = R.mgn_forward(p, x, ea, t["edge_index"], cfg)
    else:
        ref = R.bsms_forward(p, x, ea, t["edge_index"], cfg, None, t["pos"].double(), stable=True)
    lref = torch.nn.functional.mse_loss(ref, y)
    lref.backward()
    model = model.to(DEV)
    if kind == "mgn":
        pred = model(x.to(DEV), ea.to(DEV), t["edge_index"].to(DEV))
    else:
        pred = model(x.to(DEV), ea.to(DEV), t["edge_index"].to(DEV), pos=t["pos"].double().to(DEV))
    assert pred.dtype == torch.float64
    loss = torch.nn.functional.mse_loss(pred, y.to(DEV))
    loss.backward()
    _check(f"{kind} pred", pred, ref, 1e-9)
    assert abs(float(loss) - float(lref)) <= 1e-9 * float(lref)
    errs = {n: rel_l2(q.grad.detach().cpu(), p[n].grad) for n, q in model.named_parameters()}
    worst = max(errs, key=errs.get)
    print(f"f64 {kind} step: param-grad rel-L2 median {np.median(list(errs.values())):.3e}, "
          f"worst {errs[worst]:.3e} ({worst})")
    assert errs[worst] <= 1e-8, (worst, errs[worst])


@pytest.mark.parametrize("method", ["mean", "max", "add"])
def test_f64_poolmgn_vs_oracle(method):
    """poolMGN (models/poolmgn.py, §8f row 4) in fp64 on a 3-mesh batch: global pooling (segment
    sums / max in float64), broadcast, encoders, 4 layers, decoder; prediction and every parameter
    gradient against the float64 oracle."""
    from aerognn.meshgen import collate, ellipsoid
    from models.poolmgn import poolMGN
    from oracle import refcpu as R
    b = collate([ellipsoid(30, 20, seed=s) for s in (0, 1)] + [ellipsoid(24, 12, seed=2)])
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    kw = dict(processor_size=4, num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
              num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
              aggregation="add", global_pool_method=method, num_hidden_layers_global_encoder=1, global_dim=128)
    torch.manual_seed(0)
    model = poolMGN(6, 4, 4, **kw).double()
    x, ea, y = t["x"].double(), t["edge_attr"].double(), t["y"].double()
    p = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    ref = R.poolmgn_forward(p, x, ea, t["edge_index"], R.cfg_from_kwargs(**kw), batch=t["batch"])
    torch.nn.functional.mse_loss(ref, y).backward()
    model = model.to(DEV)
    pred = model(x.to(DEV), ea.to(DEV), t["edge_index"].to(DEV), batch=t["batch"].to(DEV))
    torch.nn.functional.mse_loss(pred, y.to(DEV)).backward()
    _check(f"poolmgn {method} pred", pred, ref, 1e-9)
    errs = {n: rel_l2(q.grad.detach().cpu(), p[n].grad) for n, q in model.named_parameters() if p[n].grad is not None}
    worst = max(errs, key=errs.get)
    print(f"f64 poolmgn {method}: param-grad rel-L2 worst {errs[worst]:.3e} ({worst})")
    assert errs[worst] <= 1e-8, (worst, errs[worst])


def test_f64_input_to_float32_model_raises():
    """a float32 MLP given a float64 input raises TypeError (as torch's mm does)
    instead of the agn_f64_* kernels reading the float32 weights as doubles."""
    from models.mlp import MLP
    m = MLP(16, 32, 8, 1, use_layer_norm=True).to(DEV)
    x = torch.randn(100, 16, dtype=torch.float64, device=DEV)
    with pytest.raises(TypeError):
        m(x)
