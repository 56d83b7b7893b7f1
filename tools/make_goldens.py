"""Generate golden input/output vectors from the REAL reference (this container only).

Imports /root/reference/models/{mlp,mgnLayer,mgn,bsms_mgn}.py after injecting two
in-memory stand-ins:
  * torch_scatter.scatter_add / scatter_mean — restated on Tensor.scatter_add_ exactly as
    torch_scatter's Python wrappers do (sum; mean = sum / clamp(count, 1), count in src dtype);
  * torch_geometric / torch_geometric.nn — names only (never called on the hot path).

Writes tests/golden/<case>.npz (tensors + a JSON meta string; no pickles). The reference
itself never travels: only these vectors do. Run:  python tools/make_goldens.py
"""
from __future__ import annotations

import json
import os
import sys
import types

# the reference tree is read-only input: never leave __pycache__ files in it when importing it
sys.dont_write_bytecode = True

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "aero-gnn_amd"))
from aerognn.meshgen import ellipsoid, collate  # noqa: E402


def _install_standins():
    ts = types.ModuleType("torch_scatter")

    def scatter_add(src, index, dim=-1, out=None, dim_size=None):
        dim = dim % src.dim()
        if dim_size is None:
            dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
        idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src) if index.dim() == 1 else index
        if out is None:
            size = list(src.shape)
            size[dim] = dim_size
            out = torch.zeros(size, dtype=src.dtype, device=src.device)
        return out.scatter_add_(dim, idx, src)

    def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
        out = scatter_add(src, index, dim, out, dim_size)
        ones = torch.ones(index.size(), dtype=src.dtype, device=src.device)
        count = scatter_add(ones, index, 0, None, out.size(dim % src.dim()))
        count[count < 1] = 1
        count = count.view(-1, *([1] * (src.dim() - 1))).expand_as(out)
        return out.true_divide_(count)

    ts.scatter_add = scatter_add
    ts.scatter_mean = scatter_mean
    ts.scatter_sum = scatter_add
    tg = types.ModuleType("torch_geometric")
    tgn = types.ModuleType("torch_geometric.nn")

    # torch_geometric.nn.global_{add,mean,max}_pool (unpinned version, not installed here), restated
    # from PyG's published algorithm: size = batch.max() + 1; torch_geometric.utils.scatter with
    # reduce 'sum' (scatter_add_), 'mean' (sum / count.clamp(min=1)), 'max' (zero-initialised
    # scatter_reduce_('amax', include_self=False)). Used only by models/poolmgn.py.
    def _pool(x, batch, reduce, size=None):
        if batch is None:
            batch = torch.zeros(x.size(0), dtype=torch.long, device=x.device)
        size = int(batch.max()) + 1 if size is None else size
        idx = batch.view(-1, 1).expand_as(x)
        out = x.new_zeros(size, x.size(1))
        if reduce == "max":
            return out.scatter_reduce_(0, idx, x, reduce="amax", include_self=False)
        out = out.scatter_add_(0, idx, x)
        if reduce == "mean":
            cnt = x.new_zeros(size).scatter_add_(0, batch, x.new_ones(x.size(0))).clamp_(min=1)
            out = out / cnt.view(-1, 1)
        return out

    tgn.global_add_pool = lambda x, batch, size=None: _pool(x, batch, "sum", size)
    tgn.global_mean_pool = lambda x, batch, size=None: _pool(x, batch, "mean", size)
    tgn.global_max_pool = lambda x, batch, size=None: _pool(x, batch, "max", size)
    tg.nn = tgn
    sys.modules["torch_scatter"] = ts
    sys.modules["torch_geometric"] = tg
    sys.modules["torch_geometric.nn"] = tgn


_install_standins()
# the reference's models/ (a namespace package: no __init__.py) must not be shadowed by this
# repo's regular package aero-gnn_amd/models, which would win the import scan
sys.path[:] = [p for p in sys.path if os.path.abspath(p) != os.path.abspath(os.path.join(os.path.dirname(__file__), "..",
                                                                                            "aero-gnn_amd"))]
sys.modules.pop("models", None)
sys.path.insert(0, REF)
from models.mlp import MLP  # noqa: E402
from models.mgnLayer import EdgeBlock, EdgeBlockSum, NodeBlock, MeshGraphNetLayer  # noqa: E402
from models.mgn import MeshGraphNet  # noqa: E402
from models.bsms_mgn import BiStridedMeshGraphNet  # noqa: E402
from models.poolmgn import poolMGN  # noqa: E402
import models.mlp as _refcheck  # noqa: E402
assert os.path.abspath(_refcheck.__file__).startswith(REF), _refcheck.__file__  # the REFERENCE's modules


def _np(t):
    return t.detach().cpu().numpy()


def save(name, meta, **arrs):
    os.makedirs(OUT, exist_ok=True)
    d = {k: (_np(v) if torch.is_tensor(v) else np.asarray(v)) for k, v in arrs.items()}
    d["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **d)
    print(f"{name}: {sum(v.nbytes for v in d.values()) / 1e3:.1f} kB raw")


def sd(m, prefix="p:"):
    return {prefix + k: v for k, v in m.state_dict().items()}


def grads(m, prefix="gp:"):
    return {prefix + k: p.grad for k, p in m.named_parameters() if p.grad is not None}


def mesh_tensors(nu, nv, seed=0, dtype=torch.float32, shuffle=False):
    m = ellipsoid(nu, nv, seed=seed)
    t = {k: torch.from_numpy(v) for k, v in m.items()}
    for k in ("x", "edge_attr", "y", "pos"):
        t[k] = t[k].to(dtype)
    if shuffle:
        g = torch.Generator().manual_seed(123 + seed)
        perm = torch.randperm(t["edge_index"].shape[1], generator=g)
        t["edge_index"] = t["edge_index"][:, perm]
        t["edge_attr"] = t["edge_attr"][perm]
    return t


def batch_tensors(specs, dtype=torch.float32):
    ms = [ellipsoid(nu, nv, seed=s) for nu, nv, s in specs]
    b = collate(ms)
    t = {k: torch.from_numpy(v) for k, v in b.items()}
    for k in ("x", "edge_attr", "y", "pos"):
        t[k] = t[k].to(dtype)
    return t


def case_mlp():
    torch.manual_seed(0)
    for nh in (0, 1, 2):
        m = MLP(6, 32, 32, num_hidden_layers=nh)
        x = torch.randn(50, 6, requires_grad=True)
        y = m(x)
        gy = torch.randn_like(y)
        y.backward(gy)
        save(f"mlp_nh{nh}", dict(input_dim=6, hidden_dim=32, output_dim=32, num_hidden_layers=nh,
                                 use_layer_norm=True),
             x=x, y=y, gy=gy, gx=x.grad, **sd(m), **grads(m))
    m = MLP(32, 32, 4, num_hidden_layers=2, use_layer_norm=False)
    x = torch.randn(50, 32, requires_grad=True)
    y = m(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    save("mlp_dec", dict(input_dim=32, hidden_dim=32, output_dim=4, num_hidden_layers=2,
                         use_layer_norm=False), x=x, y=y, gy=gy, gx=x.grad, **sd(m), **grads(m))


def case_layer(name, H, nu, nv, trick, agg="add", nh=2, shuffle=False, dtype=torch.float32, act="relu"):
    torch.manual_seed(1)
    t = mesh_tensors(nu, nv, shuffle=shuffle)
    N, E = t["x"].shape[0], t["edge_index"].shape[1]
    layer = MeshGraphNetLayer(H, H, H, nh, nh, act, True, agg, trick).to(dtype)
    x = torch.randn(N, H, dtype=dtype, requires_grad=True)
    e = torch.randn(E, H, dtype=dtype, requires_grad=True)
    ei = t["edge_index"]
    xo, eo = layer(x, e, ei)
    gx = torch.randn_like(xo)
    ge = torch.randn_like(eo)
    torch.autograd.backward([xo, eo], [gx, ge])
    meta = dict(H=H, trick=trick, aggregation=agg, n_hid=nh, dtype=str(dtype), activation_fn=act)
    save(name, meta, x=x, e=e, edge_index=ei, x_out=xo, e_out=eo, gx_out=gx, ge_out=ge,
         gx=x.grad, ge=e.grad, **sd(layer), **grads(layer))


def case_act():
    """activation_fn gelu / silu / tanh (mlp.py:37 getattr(F, activation_fn)): an MLP per activation
    at H = 128; concat-EdgeBlock layers (both chains take the activation) and a sum-trick layer (its
    edge chain stays ReLU, mgnLayer.py:81; the node chain takes it); a float64 layer with GELU."""
    for act in ("gelu", "silu", "tanh"):
        torch.manual_seed(9)
        m = MLP(6, 128, 128, num_hidden_layers=2, activation_fn=act)
        x = torch.randn(70, 6, requires_grad=True)
        y = m(x)
        gy = torch.randn_like(y)
        y.backward(gy)
        save(f"mlp_{act}_h128", dict(input_dim=6, hidden_dim=128, output_dim=128, num_hidden_layers=2,
                                     use_layer_norm=True, activation_fn=act),
             x=x, y=y, gy=gy, gx=x.grad, **sd(m), **grads(m))
    case_layer("layer_cat_h128_gelu", 128, 8, 6, False, shuffle=True, act="gelu")
    case_layer("layer_sum_h32_silu", 32, 10, 6, True, act="silu")
    case_layer("layer_cat_h32_tanh", 32, 10, 6, False, shuffle=True, act="tanh")
    case_layer("layer_sum_h32_f64_gelu", 32, 10, 6, True, dtype=torch.float64, act="gelu")


def case_blocks():
    torch.manual_seed(2)
    H = 32
    t = mesh_tensors(12, 8, shuffle=True)
    N, E = t["x"].shape[0], t["edge_index"].shape[1]
    ei = t["edge_index"]
    x = torch.randn(N, H, requires_grad=True)
    e = torch.randn(E, H, requires_grad=True)
    for cls, nm in ((EdgeBlockSum, "edgeblocksum"), (EdgeBlock, "edgeblock")):
        x.grad = None
        e.grad = None
        blk = cls(H, H, H, 2, "relu", True)
        y = blk(e, x, ei)
        gy = torch.randn_like(y)
        y.backward(gy)
        save(nm, dict(H=H, n_hid=2), x=x, e=e, edge_index=ei, y=y, gy=gy, gx=x.grad, ge=e.grad,
             **sd(blk), **grads(blk))
    for agg in ("add", "mean"):
        x.grad = None
        e.grad = None
        blk = NodeBlock(H, H, H, 2, "relu", True, agg)
        y = blk(x, e, ei)
        gy = torch.randn_like(y)
        y.backward(gy)
        save(f"nodeblock_{agg}", dict(H=H, n_hid=2, aggregation=agg), x=x, e=e, edge_index=ei,
             y=y, gy=gy, gx=x.grad, ge=e.grad, **sd(blk), **grads(blk))


MODEL_KW = dict(activation_fn="relu", num_hidden_layers_node_processor=2,
                num_hidden_layers_edge_processor=2, hidden_dim_processor=32,
                num_hidden_layers_node_encoder=2, hidden_dim_node_encoder=32,
                num_hidden_layers_edge_encoder=2, hidden_dim_edge_encoder=32,
                aggregation="add", hidden_dim_decoder=32, num_hidden_layers_decoder=2,
                dropout=0.0, do_concat_trick=True)


def case_mgn(dtype, name):
    torch.manual_seed(3)
    t = mesh_tensors(12, 8, dtype=dtype)
    kw = dict(MODEL_KW, processor_size=5)
    m = MeshGraphNet(6, 4, 4, **kw).to(dtype)
    pred = m(t["x"], t["edge_attr"], t["edge_index"])
    loss = torch.nn.MSELoss()(pred, t["y"])
    loss.backward()
    save(name, dict(kwargs=kw, dims=[6, 4, 4], dtype=str(dtype)), x=t["x"], edge_attr=t["edge_attr"],
         edge_index=t["edge_index"], y=t["y"], pred=pred, loss=loss, **sd(m), **grads(m))


def case_bsms(name, S, P, specs, shuffle_first=False, dtype=torch.float32, stride=2, lps=2):
    torch.manual_seed(4)
    t = batch_tensors(specs, dtype)
    if shuffle_first:
        g = torch.Generator().manual_seed(7)
        perm = torch.randperm(t["edge_index"].shape[1], generator=g)
        t["edge_index"] = t["edge_index"][:, perm]
        t["edge_attr"] = t["edge_attr"][perm]
    kw = dict(MODEL_KW, processor_size=P, num_scales=S, layers_per_scale=lps, stride=stride)
    m = BiStridedMeshGraphNet(6, 4, 4, **kw).to(dtype)
    pred = m(t["x"], t["edge_attr"], t["edge_index"], batch=t["batch"], pos=t["pos"])
    loss = torch.nn.MSELoss()(pred, t["y"])
    loss.backward()
    save(name, dict(kwargs=kw, dims=[6, 4, 4], dtype=str(dtype)), x=t["x"], edge_attr=t["edge_attr"],
         edge_index=t["edge_index"], batch=t["batch"], pos=t["pos"], y=t["y"], pred=pred, loss=loss,
         **sd(m), **grads(m))


def case_downsample():
    torch.manual_seed(5)
    H = 32
    for name, specs, stride in (("downsample_2g", [(12, 8, 0), (7, 5, 1)], 2),
                                ("downsample_s3", [(9, 7, 2), (12, 8, 3), (5, 5, 4)], 3)):
        t = batch_tensors(specs)
        N, E = t["x"].shape[0], t["edge_index"].shape[1]
        m = BiStridedMeshGraphNet(6, 4, 4, hidden_dim_processor=H, stride=stride)
        node = torch.randn(N, H)
        edge = torch.randn(E, H)
        out = m._downsample(node, edge, t["edge_index"], t["batch"], t["pos"])
        cn, ce, cei, cb, cp, f2c = out
        # second level on the coarse graph
        node2 = torch.randn(cn.shape[0], H)
        out2 = m._downsample(node2, ce, cei, cb, cp)
        save(name, dict(stride=stride, H=H), node=node, edge=edge, edge_index=t["edge_index"],
             batch=t["batch"], pos=t["pos"], c_node=cn, c_edge=ce, c_edge_index=cei, c_batch=cb,
             c_pos=cp, f2c=f2c, node2=node2, c2_node=out2[0], c2_edge=out2[1],
             c2_edge_index=out2[2], c2_batch=out2[3], c2_pos=out2[4], f2c2=out2[5])
    # no-pos variant (node-order pooling) and tied x (documents reference tie order, not gated)
    t = batch_tensors([(12, 8, 0)])
    m = BiStridedMeshGraphNet(6, 4, 4, hidden_dim_processor=H, stride=2)
    node = torch.randn(t["x"].shape[0], H)
    edge = torch.randn(t["edge_index"].shape[1], H)
    out = m._downsample(node, edge, t["edge_index"], t["batch"], None)
    save("downsample_nopos", dict(stride=2, H=H), node=node, edge=edge, edge_index=t["edge_index"],
         batch=t["batch"], c_node=out[0], c_edge=out[1], c_edge_index=out[2], c_batch=out[3],
         f2c=out[5])
    mt = ellipsoid(60, 40, unique_x=False)
    pos = torch.from_numpy(mt["pos"])
    ei = torch.from_numpy(mt["edge_index"])
    N = pos.shape[0]
    out = m._downsample(torch.zeros(N, 1), torch.zeros(ei.shape[1], 1), ei,
                        torch.zeros(N, dtype=torch.long), pos)
    save("downsample_tied", dict(stride=2, note="tied x: reference unstable-argsort order, NOT gated"),
         pos=pos, edge_index=ei, f2c=out[5], c_edge_index=out[2])


def case_bf16():
    torch.manual_seed(6)
    t = mesh_tensors(12, 8)
    H = 32
    layer = MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True)
    x = torch.randn(t["x"].shape[0], H)
    e = torch.randn(t["edge_index"].shape[1], H)
    xo, eo = layer(x, e, t["edge_index"])
    lb = MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True)
    lb.load_state_dict(layer.state_dict())
    lb = lb.to(torch.bfloat16)
    xb, eb = lb(x.bfloat16(), e.bfloat16(), t["edge_index"])
    save("layer_bf16", dict(H=H, n_hid=2, trick=True), x=x, e=e, edge_index=t["edge_index"],
         x_out=xo, e_out=eo, x_out_bf16=xb.float(), e_out_bf16=eb.float(), **sd(layer))


def case_fp16():
    """The reference's fp16 mode (train.py:35-38: default dtype float16, so fp16 parameters):
    the same layer as case_bf16 cast with .half(), H = 32 and H = 128."""
    for H in (32, 128):
        torch.manual_seed(6)
        t = mesh_tensors(12, 8)
        layer = MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True)
        x = torch.randn(t["x"].shape[0], H)
        e = torch.randn(t["edge_index"].shape[1], H)
        xo, eo = layer(x, e, t["edge_index"])
        lh = MeshGraphNetLayer(H, H, H, 2, 2, "relu", True, "add", True)
        lh.load_state_dict(layer.state_dict())
        lh = lh.to(torch.float16)
        xh, eh = lh(x.half(), e.half(), t["edge_index"])
        save(f"layer_fp16_h{H}", dict(H=H, n_hid=2, trick=True), x=x, e=e, edge_index=t["edge_index"],
             x_out=xo, e_out=eo, x_out_fp16=xh.float(), e_out_fp16=eh.float(), **sd(layer))


def case_poolmgn():
    """poolMGN (models/poolmgn.py) for each global pooling method on a 2-graph batch, H = 32."""
    for method in ("mean", "max", "add"):
        torch.manual_seed(8)
        t = batch_tensors([(12, 8, 0), (10, 6, 1)])
        kw = dict(MODEL_KW, processor_size=3, aggregation="add", global_pool_method=method,
                  num_hidden_layers_global_encoder=1, global_dim=32)
        kw.pop("do_concat_trick", None)
        for k in ("num_scales", "layers_per_scale", "stride"):
            kw.pop(k, None)
        m = poolMGN(6, 4, 4, **kw)
        pred = m(t["x"], t["edge_attr"], t["edge_index"], batch=t["batch"])
        loss = torch.nn.MSELoss()(pred, t["y"])
        loss.backward()
        save(f"poolmgn_{method}", dict(kwargs=kw, dims=[6, 4, 4]), x=t["x"], edge_attr=t["edge_attr"],
             edge_index=t["edge_index"], batch=t["batch"], y=t["y"], pred=pred, loss=loss, **sd(m), **grads(m))


if __name__ == "__main__":
    torch.set_num_threads(8)
    if len(sys.argv) > 1:  # selected cases only, e.g. `python tools/make_goldens.py poolmgn`
        for c in sys.argv[1:]:
            globals()[f"case_{c}"]()
        sys.exit(0)
    case_mlp()
    case_blocks()
    case_layer("layer_sum_h32", 32, 10, 6, True)
    case_layer("layer_sum_h32_shuf", 32, 10, 6, True, shuffle=True)
    case_layer("layer_cat_h32", 32, 10, 6, False, shuffle=True)
    case_layer("layer_mean_h32", 32, 10, 6, True, agg="mean")
    case_layer("layer_sum_h128", 128, 8, 6, True)
    case_layer("layer_sum_h32_nh1", 32, 10, 6, True, nh=1)
    case_layer("layer_sum_h32_f64", 32, 10, 6, True, dtype=torch.float64)
    case_mgn(torch.float32, "mgn5_f32")
    case_mgn(torch.float64, "mgn5_f64")
    case_bsms("bsms_s3", 3, 7, [(12, 8, 0), (12, 8, 1)])
    case_bsms("bsms_s4", 4, 13, [(12, 8, 0), (9, 7, 1)], shuffle_first=True)
    case_bsms("bsms_s2_st3", 2, 5, [(10, 6, 2), (8, 5, 3), (6, 6, 4)], stride=3, lps=1)
    case_bsms("bsms_s1", 1, 4, [(12, 8, 0)])
    case_downsample()
    case_bf16()
    case_fp16()
    case_act()
