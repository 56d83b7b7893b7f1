"""Pin the oracle (oracle/refcpu.py) against golden vectors produced by the real reference.

CPU only. The oracle issues the same aten ops in the same order as the reference, so
forward outputs are expected bitwise equal; gradients through index_put_(accumulate)
are not bitwise repeatable in torch itself, so they are checked at 1e-6.
"""
import pytest
import torch

from golden_util import load, params, rel_l2
from oracle import refcpu as R

FWD_TOL = 1e-6
GRAD_TOL = 1e-5


def _leaf(p):
    return {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in p.items()}


def _check_grads(p, d, tol=GRAD_TOL):
    for k, v in p.items():
        g = d.get("gp:" + k)
        if g is None:
            continue
        assert v.grad is not None, k
        assert rel_l2(v.grad, g) <= tol, (k, rel_l2(v.grad, g))


@pytest.mark.parametrize("name", ["mlp_nh0", "mlp_nh1", "mlp_nh2", "mlp_dec", "mlp_gelu_h128", "mlp_silu_h128",
                                  "mlp_tanh_h128"])
def test_mlp(name):
    d, m = load(name)
    p = _leaf(params(d))
    x = d["x"].clone().requires_grad_(True)
    nlin = R.mlp_nlin(m["num_hidden_layers"])
    # MLP state dict keys have no module prefix: "layers.0.weight"
    pp = {"m." + k: v for k, v in p.items()}
    y = R.mlp(pp, "m", x, nlin, ln=m["use_layer_norm"], act=R.act_of(m))
    assert torch.equal(y, d["y"]) or rel_l2(y, d["y"]) <= FWD_TOL
    y.backward(d["gy"])
    assert rel_l2(x.grad, d["gx"]) <= GRAD_TOL
    _check_grads({k[2:]: v for k, v in pp.items()}, d)


@pytest.mark.parametrize("name,kind", [("edgeblocksum", "sum"), ("edgeblock", "cat"),
                                       ("nodeblock_add", "add"), ("nodeblock_mean", "mean")])
def test_blocks(name, kind):
    d, m = load(name)
    p = {"b." + k: v for k, v in _leaf(params(d)).items()}
    x = d["x"].clone().requires_grad_(True)
    e = d["e"].clone().requires_grad_(True)
    ei = d["edge_index"]
    if kind == "sum":
        y = R.edge_block_sum(p, "b", e, x, ei, m["n_hid"])
    elif kind == "cat":
        y = R.edge_block_cat(p, "b", e, x, ei, m["n_hid"])
    else:
        y = R.node_block(p, "b", x, e, ei, m["n_hid"], kind)
    assert rel_l2(y, d["y"]) <= FWD_TOL
    y.backward(d["gy"])
    assert rel_l2(x.grad, d["gx"]) <= GRAD_TOL
    assert rel_l2(e.grad, d["ge"]) <= GRAD_TOL
    _check_grads({k[2:]: v for k, v in p.items()}, d)


LAYERS = ["layer_sum_h32", "layer_sum_h32_shuf", "layer_cat_h32", "layer_mean_h32",
          "layer_sum_h128", "layer_sum_h32_nh1", "layer_sum_h32_f64",
          "layer_cat_h128_gelu", "layer_sum_h32_silu", "layer_cat_h32_tanh", "layer_sum_h32_f64_gelu"]


@pytest.mark.parametrize("name", LAYERS)
def test_layer(name):
    d, m = load(name)
    p = {"L." + k: v for k, v in _leaf(params(d)).items()}
    x = d["x"].clone().requires_grad_(True)
    e = d["e"].clone().requires_grad_(True)
    cfg = dict(do_concat_trick=m["trick"], n_hid_edge=m["n_hid"], n_hid_node=m["n_hid"],
               aggregation=m["aggregation"], activation_fn=m.get("activation_fn", "relu"))
    xo, eo = R.gmp_layer(p, "L", x, e, d["edge_index"], cfg)
    assert torch.equal(xo, d["x_out"]) or rel_l2(xo, d["x_out"]) <= FWD_TOL
    assert torch.equal(eo, d["e_out"]) or rel_l2(eo, d["e_out"]) <= FWD_TOL
    torch.autograd.backward([xo, eo], [d["gx_out"], d["ge_out"]])
    assert rel_l2(x.grad, d["gx"]) <= GRAD_TOL
    assert rel_l2(e.grad, d["ge"]) <= GRAD_TOL
    _check_grads({k[2:]: v for k, v in p.items()}, d)


@pytest.mark.parametrize("name", ["layer_bf16", "layer_fp16_h32", "layer_fp16_h128"])
def test_layer_16bit_modes(name):
    """The reference's bf16 / fp16 modes (train.py:30-38: 16-bit parameters and activations): the
    oracle, run with the golden's parameters cast to that dtype, reproduces the reference's
    16-bit outputs bitwise, and its fp32 outputs bitwise in fp32."""
    d, m = load(name)
    dt, suffix = (torch.bfloat16, "bf16") if name == "layer_bf16" else (torch.float16, "fp16")
    p = {"L." + k: v for k, v in params(d).items()}
    cfg = dict(do_concat_trick=m["trick"], n_hid_edge=m["n_hid"], n_hid_node=m["n_hid"], aggregation="add")
    xo, eo = R.gmp_layer(p, "L", d["x"], d["e"], d["edge_index"], cfg)
    assert torch.equal(xo, d["x_out"]) and torch.equal(eo, d["e_out"])
    ph = {k: v.to(dt) for k, v in p.items()}
    xh, eh = R.gmp_layer(ph, "L", d["x"].to(dt), d["e"].to(dt), d["edge_index"], cfg)
    assert torch.equal(xh.float(), d[f"x_out_{suffix}"]) and torch.equal(eh.float(), d[f"e_out_{suffix}"])


@pytest.mark.parametrize("name", ["mgn5_f32", "mgn5_f64"])
def test_mgn(name):
    d, m = load(name)
    p = _leaf(params(d))
    cfg = R.cfg_from_kwargs(**m["kwargs"])
    pred = R.mgn_forward(p, d["x"], d["edge_attr"], d["edge_index"], cfg)
    assert rel_l2(pred, d["pred"]) <= FWD_TOL
    loss = torch.nn.functional.mse_loss(pred, d["y"])
    loss.backward()
    _check_grads(p, d)


@pytest.mark.parametrize("name", ["bsms_s3", "bsms_s4", "bsms_s2_st3", "bsms_s1"])
def test_bsms(name):
    d, m = load(name)
    p = _leaf(params(d))
    cfg = R.cfg_from_kwargs(**m["kwargs"])
    pred = R.bsms_forward(p, d["x"], d["edge_attr"], d["edge_index"], cfg, d["batch"], d["pos"],
                          stable=True)
    assert rel_l2(pred, d["pred"]) <= FWD_TOL
    loss = torch.nn.functional.mse_loss(pred, d["y"])
    loss.backward()
    _check_grads(p, d)


@pytest.mark.parametrize("name", ["downsample_2g", "downsample_s3"])
def test_downsample(name):
    d, m = load(name)
    cn, ce, cei, cb, cp, f2c = R.downsample(d["node"], d["edge"], d["edge_index"], d["batch"],
                                            d["pos"], m["stride"], stable=True)
    assert torch.equal(f2c, d["f2c"])
    assert torch.equal(cei, d["c_edge_index"])
    assert torch.equal(cb, d["c_batch"])
    assert torch.equal(cn, d["c_node"])
    assert torch.equal(ce, d["c_edge"])
    assert torch.equal(cp, d["c_pos"])
    o2 = R.downsample(d["node2"], ce, cei, cb, cp, m["stride"], stable=True)
    for got, key in zip(o2, ["c2_node", "c2_edge", "c2_edge_index", "c2_batch", "c2_pos", "f2c2"]):
        assert torch.equal(got, d[key]), key


def test_downsample_nopos():
    d, m = load("downsample_nopos")
    cn, ce, cei, cb, cp, f2c = R.downsample(d["node"], d["edge"], d["edge_index"], d["batch"],
                                            None, m["stride"])
    assert torch.equal(f2c, d["f2c"]) and torch.equal(cei, d["c_edge_index"])
    assert torch.equal(cn, d["c_node"]) and torch.equal(ce, d["c_edge"])


@pytest.mark.parametrize("method", ["mean", "max", "add"])
def test_poolmgn(method):
    """poolMGN (models/poolmgn.py) with the restated torch_geometric global pools."""
    d, m = load(f"poolmgn_{method}")
    p = _leaf(params(d))
    cfg = R.cfg_from_kwargs(**m["kwargs"])
    pred = R.poolmgn_forward(p, d["x"], d["edge_attr"], d["edge_index"], cfg, d["batch"])
    assert torch.equal(pred, d["pred"]) or rel_l2(pred, d["pred"]) <= FWD_TOL
    torch.nn.functional.mse_loss(pred, d["y"]).backward()
    _check_grads(p, d)
