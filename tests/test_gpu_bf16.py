"""bf16 training numerics against the float64 oracle.

The headline configuration trains with bf16 activations and fp32 master weights. Its backward runs
on kernels the fp32 oracle tests never reach: the fused edge backward (agn_edge_bwd_fused, bf16
H=128 sum-trick chains of >= 65,536 edges) and the bf16 instantiations of the split path. Here the
bf16 outputs and gradients are compared with the float64 CPU oracle (oracle/refcpu.py, the
reference's aten sequence, mgnLayer.py:93-105,205 / bsms_mgn.py:126-215 under autograd) on the same
fp32 weights and the same bf16-rounded inputs. bf16 rounds every activation to 8 significant bits,
so the errors are ~1e-2 and not a parity bar: each gate is 3x the value measured on the MI355X
(printed), a regression gate that a rounding bug shared by both bf16 backward paths
(e.g. a gradient rounded to bf16 at the wrong point) would trip.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"

# rel-L2 against the float64 oracle measured on the MI355X (profiles/r4_gpu_bf16_tests.log); each
# gate is 3x its value, floor 1e-6. The ReLU-masked quantities sit at 3e-2..1e-1: bf16 forward
# errors (~4e-3 of a pre-activation's scale) put ~0.2 % of the ReLU inputs on the other side of 0
# than in float64, and each such flip changes its gradient element by O(1), so the rel-L2 is about
# the square root of the flipped fraction (~5e-2 per ReLU layer). Quantities no ReLU mask reaches in
# the backward (the node MLP's last Linear and LayerNorm) show the plain bf16 rounding, ~4e-3.
C2_MEASURED = {
    "x'": 3.711e-03, "e'": 2.924e-03, "dx": 5.922e-02, "de": 2.684e-02,
    "edge_block.edge_lin": 7.848e-02, "edge_block.src_lin": 7.850e-02, "edge_block.dst_lin": 7.542e-02,
    "edge_block.bias": 7.845e-02, "edge_block.mlp.1.weight": 6.872e-02, "edge_block.mlp.1.bias": 6.697e-02,
    "edge_block.mlp.3.weight": 5.158e-02, "edge_block.mlp.3.bias": 5.221e-02, "edge_block.mlp.5.weight": 2.593e-02,
    "edge_block.mlp.5.bias": 2.921e-02, "edge_block.mlp.6.weight": 2.912e-02, "edge_block.mlp.6.bias": 2.939e-02,
    "node_block.mlp.layers.0.weight": 9.249e-02, "node_block.mlp.layers.0.bias": 9.716e-02,
    "node_block.mlp.layers.1.weight": 7.568e-02, "node_block.mlp.layers.1.bias": 7.788e-02,
    "node_block.mlp.layers.2.weight": 5.264e-02, "node_block.mlp.layers.2.bias": 5.306e-02,
    "node_block.mlp.layers.3.weight": 4.543e-03, "node_block.mlp.layers.3.bias": 2.088e-03,
    "node_block.mlp.layer_norm.weight": 3.892e-03, "node_block.mlp.layer_norm.bias": 1.119e-07,
}
# BSMS-4 bf16 steps, measured (r4j): 6,000 nodes median 2.295e-2 / worst 4.011e-2; 16,500 nodes
# 1.948e-2 / 3.723e-2; C3 (vs fp32 HIP) 1.784e-2 / 2.871e-2. Gates 3x the largest.
STEP_GATES = {"median": 6.9e-2, "worst": 1.2e-1}


def _gate(name):
    return max(3.0 * C2_MEASURED[name], 1e-6)


def _mesh(nu, nv, seed=0):
    from aerognn.meshgen import ellipsoid
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=seed).items()}


def test_c2_layer_bf16_fwd_bwd_vs_fp64_oracle():
    """One sum-trick MeshGraphNetLayer at C2 size (100,000 nodes / 598,400 edges) in bf16: the
    training backward runs agn_edge_bwd_fused. x', e', dx, de and every parameter gradient against
    the float64 oracle."""
    from aerognn import core
    from models.mgnLayer import MeshGraphNetLayer
    from oracle import refcpu as R
    m = _mesh(400, 250)
    N, E = m["x"].shape[0], m["edge_index"].shape[1]
    assert core.fused_edge_train_ok(E, torch.bfloat16, 128, 4, True)
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True)
    g = torch.Generator(device="cpu").manual_seed(4)
    x = torch.randn(N, 128, generator=g).bfloat16()
    e = torch.randn(E, 128, generator=g).bfloat16()
    gxo = torch.randn(N, 128, generator=g).bfloat16()
    geo = torch.randn(E, 128, generator=g).bfloat16()
    p = {f"L.{k}": v.double().requires_grad_(True) for k, v in layer.state_dict().items()}
    cfg = R.cfg_from_kwargs(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                            do_concat_trick=True, aggregation="add")
    ei = m["edge_index"]
    xr_in, er_in = x.double().requires_grad_(True), e.double().requires_grad_(True)
    xr, er = R.gmp_layer(p, "L", xr_in, er_in, ei, cfg)
    torch.autograd.backward([xr, er], [gxo.double(), geo.double()])
    layer = layer.to(DEV)
    xg, eg = x.to(DEV).requires_grad_(True), e.to(DEV).requires_grad_(True)
    xo, eo = layer(xg, eg, ei.to(DEV))
    assert xo.dtype == torch.bfloat16
    torch.autograd.backward([xo, eo], [gxo.to(DEV), geo.to(DEV)])
    torch.cuda.synchronize()
    fails = []
    for name, got, ref in [("x'", xo, xr), ("e'", eo, er), ("dx", xg.grad, xr_in.grad), ("de", eg.grad, er_in.grad)]:
        r = rel_l2(got.detach().cpu().double(), ref.detach())
        print(f"C2 bf16 layer {name}: rel-L2 {r:.3e} (gate {_gate(name):.2e})")
        if not r <= _gate(name):
            fails.append((name, r))
    for n, q in layer.named_parameters():
        r = rel_l2(q.grad.detach().cpu().double(), p[f"L.{n}"].grad)
        print(f"C2 bf16 layer d{n}: rel-L2 {r:.3e} (gate {_gate(n):.2e})")
        if not r <= _gate(n):
            fails.append((n, r))
    assert not fails, fails


@pytest.mark.parametrize("nu,nv", [(80, 75), (150, 110)])
def test_bsms4_bf16_train_step_grads_vs_fp64_oracle(nu, nv):
    """A whole BSMS-4 train step (the C3 architecture: 15 processor layers, H=128, sum trick) in
    bf16 on a 6,000-node mesh (every level below 65,536 edges: the split bf16 backward) and a
    16,500-node mesh (98,400 edges: every level on the fused edge backward). The distribution of
    per-parameter gradient rel-L2 against the float64 oracle (median and worst), and the loss."""
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    t = _mesh(nu, nv)
    kw = dict(processor_size=15, num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
              num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
              hidden_dim_processor=128, hidden_dim_node_encoder=128, hidden_dim_edge_encoder=128,
              hidden_dim_decoder=128, aggregation="add", do_concat_trick=True, num_scales=4, layers_per_scale=2,
              stride=2)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    x, ea = t["x"].bfloat16(), t["edge_attr"].bfloat16()
    pred = model(x.to(DEV), ea.to(DEV), t["edge_index"].to(DEV), pos=t["pos"].to(DEV))
    loss = torch.nn.functional.mse_loss(pred.float(), t["y"].to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    p64 = {k: v.detach().cpu().double().requires_grad_(True) for k, v in model.state_dict().items()}
    r64 = R.bsms_forward(p64, x.double(), ea.double(), t["edge_index"], R.cfg_from_kwargs(**kw), None,
                         t["pos"].double(), stable=True)
    l64 = torch.nn.functional.mse_loss(r64, t["y"].double())
    l64.backward()
    errs = {n: rel_l2(q.grad.detach().cpu().double(), p64[n].grad) for n, q in model.named_parameters()}
    v = np.array(list(errs.values()))
    worst = max(errs, key=errs.get)
    lrel = abs(float(loss.detach()) - float(l64.detach())) / float(l64.detach())
    print(f"BSMS-4 bf16 step on {t['x'].shape[0]} nodes / {t['edge_index'].shape[1]} edges: param-grad rel-L2 "
          f"median {np.median(v):.3e}, worst {v.max():.3e} ({worst}); loss rel err {lrel:.2e}")
    assert np.isfinite(v).all()
    assert np.median(v) <= STEP_GATES["median"] and v.max() <= STEP_GATES["worst"], (np.median(v), v.max(), worst)
    assert lrel <= 1e-2


def test_c3_bf16_train_step_grads_vs_fp32_hip():
    """The headline configuration itself (C3: 1,000,000 nodes / 5,996,000 edges, BSMS-4, 15
    processor layers): the bf16 train step's parameter gradients and loss against the fp32 HIP
    step on the same fp32 weights and the same bf16-rounded inputs. The fp32 path is pinned to the
    float64 oracle at 1e-5 on every kernel it runs (tests/test_gpu_parity.py, test_gpu_configs.py,
    the C2 layer above); at 1M nodes the CPU oracle is out of reach, so fp32 HIP stands in for it
    here, under the same distribution gates as the oracle-checked steps above."""
    from models.bsms_mgn import BiStridedMeshGraphNet
    t = {k: v.to(DEV) for k, v in _mesh(1000, 1000).items()}
    kw = dict(processor_size=15, num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
              num_hidden_layers_node_encoder=2, num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
              do_concat_trick=True, num_scales=4, layers_per_scale=2, stride=2)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw).to(DEV)
    x, ea = t["x"].bfloat16(), t["edge_attr"].bfloat16()
    res = []
    for dt in (torch.bfloat16, torch.float32):
        model.zero_grad(set_to_none=True)
        pred = model(x.to(dt), ea.to(dt), t["edge_index"], batch=None, pos=t["pos"])
        loss = torch.nn.functional.mse_loss(pred.float(), t["y"])
        loss.backward()
        torch.cuda.synchronize()
        res.append((float(loss.detach()), {n: q.grad.detach().double() for n, q in model.named_parameters()}))
    (lb, gb), (lf, gf) = res
    errs = {n: rel_l2(gb[n], gf[n]) for n in gf}
    v = np.array(list(errs.values()))
    worst = max(errs, key=errs.get)
    lrel = abs(lb - lf) / lf
    print(f"C3 bf16 step vs fp32 HIP: param-grad rel-L2 median {np.median(v):.3e}, worst {v.max():.3e} ({worst}); "
          f"loss rel err {lrel:.2e}")
    assert np.isfinite(v).all()
    assert np.median(v) <= STEP_GATES["median"] and v.max() <= STEP_GATES["worst"], (np.median(v), v.max(), worst)
    assert lrel <= 1e-2
