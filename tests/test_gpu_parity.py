"""GPU parity: the libaerognn path (drop-in models/*) vs golden vectors of the real reference
and vs the CPU oracle. fp32 bar: rel-L2 <= 1e-5 and max|err| <= 1e-5*max|ref|
per output tensor; index maps bit-exact. Gradients: rel-L2 <= 1e-5 (input grads) and
<= 5e-5 (parameter grads: sums over all rows in a different order than torch's CPU GEMMs).
"""
import os

import numpy as np
import pytest
import torch

from golden_util import load, max_rel, params, rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")

FWD = 1e-5
GIN = 1e-5
GPAR = 5e-5
DEV = "cuda"


def _lib_loaded():
    from aerognn import _lib
    _lib.lib()


def _fwd_ok(got, ref, tol=FWD):
    """SURVEY §8 fp32 bar, both parts: rel-L2 <= tol and max|err| <= tol * max|ref|."""
    got = got.detach().float().cpu()
    ref = ref.float()
    r, m = rel_l2(got, ref), max_rel(got, ref)
    print(f"fwd rel-L2 {r:.2e}, max-elem {m:.2e} (of max|ref|)")
    assert r <= tol and m <= tol, (r, m)


def _load(model, d):
    sd = {k: v for k, v in params(d).items()}
    model.load_state_dict(sd)
    return model.to(DEV)


def _check_param_grads(model, d, tol=GPAR):
    worst = ("", 0.0)
    for name, p in model.named_parameters():
        g = d.get("gp:" + name)
        if g is None:
            continue
        assert p.grad is not None, name
        r = rel_l2(p.grad.float().cpu(), g.float())
        if r > worst[1]:
            worst = (name, r)
    assert worst[1] <= tol, worst


# ------------------------------------------------------------------------------ MLP
@pytest.mark.parametrize("name", ["mlp_nh0", "mlp_nh1", "mlp_nh2", "mlp_dec", "mlp_gelu_h128", "mlp_silu_h128",
                                  "mlp_tanh_h128"])
def test_mlp(name):
    """MLP (mlp.py:40-51), including activation_fn gelu / silu / tanh (mlp.py:37) at H = 128."""
    from models.mlp import MLP
    d, m = load(name)
    model = _load(MLP(m["input_dim"], m["hidden_dim"], m["output_dim"], m["num_hidden_layers"],
                      activation_fn=m.get("activation_fn", "relu"), use_layer_norm=m["use_layer_norm"]), d)
    x = d["x"].to(DEV).requires_grad_(True)
    y = model(x)
    _fwd_ok(y, d["y"])
    y.backward(d["gy"].to(DEV))
    assert rel_l2(x.grad.cpu(), d["gx"]) <= GIN
    _check_param_grads(model, d)


@pytest.mark.parametrize("act", ["gelu", "silu", "tanh"])
def test_mlp_activation_bf16(act):
    """bf16 parameters and activations (train.py:30-34) with a non-ReLU activation_fn, against the
    reference's fp32 fixture: SURVEY §8's bf16 bar (rel-L2 <= 2e-2) on y, dx and every weight grad."""
    from models.mlp import MLP
    d, m = load(f"mlp_{act}_h128")
    model = _load(MLP(m["input_dim"], m["hidden_dim"], m["output_dim"], m["num_hidden_layers"],
                      activation_fn=act, use_layer_norm=m["use_layer_norm"]), d).to(torch.bfloat16)
    x = d["x"].to(DEV, torch.bfloat16).requires_grad_(True)
    y = model(x)
    y.backward(d["gy"].to(DEV, torch.bfloat16))
    worst = max([rel_l2(y.float().cpu(), d["y"]), rel_l2(x.grad.float().cpu(), d["gx"])] +
                [rel_l2(q.grad.float().cpu(), d["gp:" + n]) for n, q in model.named_parameters()])
    print(f"bf16 MLP {act}: worst rel-L2 {worst:.2e} against the fp32 reference")
    assert worst <= 2e-2


# ------------------------------------------------------------------------------ blocks
@pytest.mark.parametrize("name", ["edgeblocksum", "edgeblock", "nodeblock_add", "nodeblock_mean"])
def test_blocks(name):
    from models.mgnLayer import EdgeBlock, EdgeBlockSum, NodeBlock
    d, m = load(name)
    H = m["H"]
    if name == "edgeblocksum":
        blk = EdgeBlockSum(H, H, H, m["n_hid"])
    elif name == "edgeblock":
        blk = EdgeBlock(H, H, H, m["n_hid"])
    else:
        blk = NodeBlock(H, H, H, m["n_hid"], aggregation=m["aggregation"])
    blk = _load(blk, d)
    x = d["x"].to(DEV).requires_grad_(True)
    e = d["e"].to(DEV).requires_grad_(True)
    ei = d["edge_index"].to(DEV)
    y = blk(e, x, ei) if name.startswith("edge") else blk(x, e, ei)
    _fwd_ok(y, d["y"])
    y.backward(d["gy"].to(DEV))
    assert rel_l2(x.grad.cpu(), d["gx"]) <= GIN, rel_l2(x.grad.cpu(), d["gx"])
    assert rel_l2(e.grad.cpu(), d["ge"]) <= GIN, rel_l2(e.grad.cpu(), d["ge"])
    _check_param_grads(blk, d)


# ------------------------------------------------------------------------------ layers
LAYERS = ["layer_sum_h32", "layer_sum_h32_shuf", "layer_cat_h32", "layer_mean_h32", "layer_sum_h128",
          "layer_sum_h32_nh1", "layer_cat_h128_gelu", "layer_sum_h32_silu", "layer_cat_h32_tanh"]


@pytest.mark.parametrize("name", LAYERS)
def test_layer(name):
    from models.mgnLayer import MeshGraphNetLayer
    d, m = load(name)
    H, nh = m["H"], m["n_hid"]
    layer = _load(MeshGraphNetLayer(H, H, H, nh, nh, m.get("activation_fn", "relu"), True, m["aggregation"],
                                    m["trick"]), d)
    x = d["x"].to(DEV).requires_grad_(True)
    e = d["e"].to(DEV).requires_grad_(True)
    xo, eo = layer(x, e, d["edge_index"].to(DEV))
    _fwd_ok(xo, d["x_out"])
    _fwd_ok(eo, d["e_out"])
    torch.autograd.backward([xo, eo], [d["gx_out"].to(DEV), d["ge_out"].to(DEV)])
    assert rel_l2(x.grad.cpu(), d["gx"]) <= GIN, rel_l2(x.grad.cpu(), d["gx"])
    assert rel_l2(e.grad.cpu(), d["ge"]) <= GIN, rel_l2(e.grad.cpu(), d["ge"])
    _check_param_grads(layer, d)


def test_layer_bf16():
    """bf16 activations vs the fp32 reference (rel-L2 <= 2e-2 per layer output)."""
    from models.mgnLayer import MeshGraphNetLayer
    d, m = load("layer_bf16")
    H = m["H"]
    layer = _load(MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True), d)
    x = d["x"].to(DEV).bfloat16()
    e = d["e"].to(DEV).bfloat16()
    with torch.no_grad():
        xo, eo = layer(x, e, d["edge_index"].to(DEV))
    assert rel_l2(xo.float().cpu(), d["x_out"]) <= 2e-2
    assert rel_l2(eo.float().cpu(), d["e_out"]) <= 2e-2


# ------------------------------------------------------------------------------ models
def _model_from(meta, cls):
    kw = dict(meta["kwargs"])
    return cls(*meta["dims"], **kw)


def test_mgn():
    from models.mgn import MeshGraphNet
    d, m = load("mgn5_f32")
    model = _load(_model_from(m, MeshGraphNet), d)
    pred = model(d["x"].to(DEV), d["edge_attr"].to(DEV), d["edge_index"].to(DEV))
    _fwd_ok(pred, d["pred"])
    loss = torch.nn.functional.mse_loss(pred, d["y"].to(DEV))
    loss.backward()
    _check_param_grads(model, d)


@pytest.mark.parametrize("name", ["bsms_s3", "bsms_s4", "bsms_s2_st3", "bsms_s1"])
def test_bsms(name):
    from models.bsms_mgn import BiStridedMeshGraphNet
    d, m = load(name)
    model = _load(_model_from(m, BiStridedMeshGraphNet), d)
    pred = model(d["x"].to(DEV), d["edge_attr"].to(DEV), d["edge_index"].to(DEV), batch=d["batch"].to(DEV),
                 pos=d["pos"].to(DEV))
    _fwd_ok(pred, d["pred"])
    loss = torch.nn.functional.mse_loss(pred, d["y"].to(DEV))
    loss.backward()
    _check_param_grads(model, d)


# ------------------------------------------------------------------------------ pooling maps
@pytest.mark.parametrize("name", ["downsample_2g", "downsample_s3"])
def test_downsample_bitexact(name):
    from models.bsms_mgn import BiStridedMeshGraphNet
    d, m = load(name)
    model = BiStridedMeshGraphNet(6, 4, 4, hidden_dim_processor=m["H"], stride=m["stride"]).to(DEV)
    out = model._downsample(d["node"].to(DEV), d["edge"].to(DEV), d["edge_index"].to(DEV), d["batch"].to(DEV),
                            d["pos"].to(DEV))
    cn, ce, cei, cb, cp, f2c = [o.cpu() for o in out]
    assert torch.equal(f2c, d["f2c"])
    assert torch.equal(cei, d["c_edge_index"])
    assert torch.equal(cb, d["c_batch"])
    assert torch.equal(cn, d["c_node"])          # fp32 means in the reference's summation order
    assert torch.equal(ce, d["c_edge"])
    assert torch.equal(cp, d["c_pos"])
    out2 = model._downsample(d["node2"].to(DEV), d["c_edge"].to(DEV), d["c_edge_index"].to(DEV),
                             d["c_batch"].to(DEV), d["c_pos"].to(DEV))
    for got, key in zip(out2, ["c2_node", "c2_edge", "c2_edge_index", "c2_batch", "c2_pos", "f2c2"]):
        assert torch.equal(got.cpu(), d[key]), key


def test_downsample_nopos():
    from models.bsms_mgn import BiStridedMeshGraphNet
    d, m = load("downsample_nopos")
    model = BiStridedMeshGraphNet(6, 4, 4, hidden_dim_processor=m["H"], stride=m["stride"]).to(DEV)
    cn, ce, cei, cb, cp, f2c = model._downsample(d["node"].to(DEV), d["edge"].to(DEV), d["edge_index"].to(DEV),
                                                 d["batch"].to(DEV), None)
    assert torch.equal(f2c.cpu(), d["f2c"]) and torch.equal(cei.cpu(), d["c_edge_index"])
    assert torch.equal(cn.cpu(), d["c_node"]) and torch.equal(ce.cpu(), d["c_edge"])


# ------------------------------------------------------------------------------ vs oracle
def _oracle_compare(kind, nu, nv, S=4, H=128, P=15, seeds=(0,), tol=FWD, grads=True, dtype=torch.float32):
    from aerognn.meshgen import collate, ellipsoid
    from oracle import refcpu as R
    b = collate([ellipsoid(nu, nv, seed=s) for s in seeds])
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    kw = dict(processor_size=P, num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
              num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
              hidden_dim_processor=H, hidden_dim_node_encoder=H, hidden_dim_edge_encoder=H, hidden_dim_decoder=H,
              aggregation="add", do_concat_trick=True)
    torch.manual_seed(0)
    if kind == "mgn":
        from models.mgn import MeshGraphNet
        model = MeshGraphNet(6, 4, 4, **kw).to(DEV)
        pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV))
    else:
        from models.bsms_mgn import BiStridedMeshGraphNet
        kw.update(num_scales=S, layers_per_scale=2, stride=2)
        model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
        pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV), batch=t["batch"].to(DEV),
                     pos=t["pos"].to(DEV))
    p = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    cfg = R.cfg_from_kwargs(**kw)
    if kind == "mgn":
        ref = R.mgn_forward(p, t["x"], t["edge_attr"], t["edge_index"], cfg)
    else:
        ref = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], cfg, t["batch"], t["pos"], stable=True)
    _fwd_ok(pred, ref.detach(), tol)
    if grads:
        # gradients of a 15-layer net are ill-conditioned: judge against an fp64 oracle, and
        # require our fp32 error to be within 10x of the fp32 CPU reference's own error
        torch.nn.functional.mse_loss(pred, t["y"].to(DEV)).backward()
        torch.nn.functional.mse_loss(ref, t["y"]).backward()
        p64 = {k: v.detach().double().requires_grad_(True) for k, v in p.items()}
        if kind == "mgn":
            r64 = R.mgn_forward(p64, t["x"].double(), t["edge_attr"].double(), t["edge_index"], cfg)
        else:
            r64 = R.bsms_forward(p64, t["x"].double(), t["edge_attr"].double(), t["edge_index"], cfg, t["batch"],
                                 t["pos"].double(), stable=True)
        torch.nn.functional.mse_loss(r64, t["y"].double()).backward()
        print(f"FWD vs fp64: ours {rel_l2(pred.detach().cpu().double(), r64.detach()):.3e} "
              f"cpu32 {rel_l2(ref.detach().double(), r64.detach()):.3e}")
        # Per parameter the fp32 error is dominated by ReLU kinks: a pre-activation within
        # rounding distance of 0 flips its mask in one fp32 evaluation and not in another, so
        # WHICH parameters carry ~1e-4..1e-3 error differs between two valid fp32 evaluation
        # orders (the CPU reference itself shows 4e-4 on some of this model's params). Gate on
        # the error distribution over all parameters instead of parameter-by-parameter.
        ours_e, cpu_e = [], []
        for n, q in model.named_parameters():
            g64 = p64[n].grad
            ours_e.append(rel_l2(q.grad.cpu().double(), g64))
            cpu_e.append(rel_l2(p[n].grad.double(), g64))
            print(f"GRAD {n:60s} ours {ours_e[-1]:.3e} cpu32 {cpu_e[-1]:.3e}")
        ours_e, cpu_e = torch.tensor(ours_e), torch.tensor(cpu_e)
        assert ours_e.max() <= 10 * max(cpu_e.max(), 1e-6), (float(ours_e.max()), float(cpu_e.max()))
        assert ours_e.median() <= 10 * max(cpu_e.median(), 1e-6), (float(ours_e.median()), float(cpu_e.median()))


def test_oracle_mgn15_c1():
    """C1: MGN-15, ellipsoid(40,25) = 1,000 nodes / 5,840 edges, H=128, fp32."""
    _oracle_compare("mgn", 40, 25)


def test_oracle_bsms4_batch():
    """BSMS S=4 on a 2-mesh batch of unequal sizes, H=128, fp32, forward + all parameter grads."""
    _oracle_compare("bsms", 30, 20, S=4, seeds=(0, 1))


# ------------------------------------------------------------------------------ properties
def test_deterministic():
    """No float atomics: two runs are bitwise identical (forward and parameter grads)."""
    from aerognn.meshgen import ellipsoid
    from models.bsms_mgn import BiStridedMeshGraphNet
    m = ellipsoid(60, 40)
    t = {k: torch.from_numpy(v).to(DEV) for k, v in m.items()}
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, num_scales=3, do_concat_trick=True).to(DEV)
    outs = []
    for _ in range(2):
        model.zero_grad()
        pred = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"])
        torch.nn.functional.mse_loss(pred, t["y"]).backward()
        outs.append((pred.detach().clone(), [p.grad.clone() for p in model.parameters()]))
    assert torch.equal(outs[0][0], outs[1][0])
    for a, b in zip(outs[0][1], outs[1][1]):
        assert torch.equal(a, b)


def test_native_lib_loaded():
    import aerognn._lib as L
    _lib_loaded()
    assert L._lib is not None


# ------------------------------------------------------------------------------ poolMGN (§8f row 4)
@pytest.mark.parametrize("method", ["mean", "max", "add"])
def test_poolmgn(method):
    """models/poolmgn.py: global encoder -> global_{mean,max,add}_pool -> broadcast -> concat ->
    MeshGraphNet, vs the reference's goldens (forward and parameter grads)."""
    from models.poolmgn import poolMGN
    d, m = load(f"poolmgn_{method}")
    model = _load(_model_from(m, poolMGN), d)
    pred = model(d["x"].to(DEV), d["edge_attr"].to(DEV), d["edge_index"].to(DEV), batch=d["batch"].to(DEV))
    _fwd_ok(pred, d["pred"])
    torch.nn.functional.mse_loss(pred, d["y"].to(DEV)).backward()
    # this golden sits on a ReLU kink: the reference's own fp32 gradient of layers.2's edge MLP is
    # 1.0e-3 from the exact (float64) one, and the HIP fp32 gradient takes the exact side. So every
    # parameter gradient is gated against the float64 oracle at max(5e-5, 10x the reference's own
    # fp32-vs-float64 error), and the golden itself at 5e-5 wherever the reference is kink-free.
    from oracle import refcpu as R
    cfg = R.cfg_from_kwargs(**m["kwargs"])
    p64 = {k: v.double().clone().requires_grad_(True) for k, v in params(d).items()}
    r64 = R.poolmgn_forward(p64, d["x"].double(), d["edge_attr"].double(), d["edge_index"], cfg, batch=d["batch"])
    torch.nn.functional.mse_loss(r64, d["y"].double()).backward()
    for name, prm in model.named_parameters():
        g32, g64 = d.get("gp:" + name), p64[name].grad
        if g32 is None or g64 is None:
            continue
        own = rel_l2(g32.double(), g64)
        err64 = rel_l2(prm.grad.double().cpu(), g64)
        assert err64 <= max(GPAR, 10 * own), (name, err64, own)
        if own <= GPAR / 10:
            assert rel_l2(prm.grad.float().cpu(), g32.float()) <= GPAR, name


@pytest.mark.parametrize("method", ["mean", "max"])
def test_poolmgn_h128_vs_oracle(method):
    """H = 128 poolMGN on a 3-mesh batch (unequal sizes) and without `batch`, vs the oracle."""
    from aerognn.meshgen import collate, ellipsoid
    from models.poolmgn import poolMGN
    from oracle import refcpu as R
    b = collate([ellipsoid(30, 20, seed=s) for s in (0, 1)] + [ellipsoid(24, 12, seed=2)])
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    kw = dict(processor_size=4, num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
              num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
              aggregation="add", global_pool_method=method, num_hidden_layers_global_encoder=1, global_dim=128)
    torch.manual_seed(0)
    model = poolMGN(6, 4, 4, **kw).to(DEV)
    p = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    cfg = R.cfg_from_kwargs(**kw)
    for batch in (t["batch"], None):
        pred = model(t["x"].to(DEV), t["edge_attr"].to(DEV), t["edge_index"].to(DEV),
                     batch=batch.to(DEV) if batch is not None else None)
        with torch.no_grad():
            ref = R.poolmgn_forward(p, t["x"], t["edge_attr"], t["edge_index"], cfg, batch)
        _fwd_ok(pred, ref)
