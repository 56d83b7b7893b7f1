"""ORACLE — test infrastructure only. Never imported by the product path.

CPU restatement (eager PyTorch, fp32/fp64 on CPU) of the reference's hot path,
op-for-op in the reference's order so that it is bitwise equal to the imported
reference on CPU. Parameters are passed as a flat dict whose keys are exactly the
reference `state_dict` keys, so the same dict loads into the
product modules (`aero-gnn_amd/models`).

Pinned by: tests/test_oracle_golden.py against tests/golden/*.npz, which
tools/make_goldens.py produced by importing /root/reference/models/* (with
in-memory torch_scatter / torch_geometric stand-ins).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

# --------------------------------------------------------------------------------------
# torch_scatter restatement (third-party, unpinned). torch_scatter.scatter_sum
# = zeros(...).scatter_add_(dim, broadcast(index), src); scatter_mean = sum / clamp(count,1)
# with count in src dtype (true_divide).
# --------------------------------------------------------------------------------------


def scatter_add(src, index, dim=0, dim_size=None):
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    size = list(src.shape)
    size[dim] = dim_size
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return torch.zeros(size, dtype=src.dtype, device=src.device).scatter_add_(dim, idx, src)


def scatter_mean(src, index, dim=0, dim_size=None):
    out = scatter_add(src, index, dim, dim_size)
    ones = torch.ones(index.size(), dtype=src.dtype, device=src.device)
    count = scatter_add(ones, index, 0, out.size(dim))
    count[count < 1] = 1
    count = count.view(-1, *([1] * (src.dim() - 1))).expand_as(out)
    return out.true_divide(count)


# --------------------------------------------------------------------------------------
# models/mlp.py:40-51  (MLP.forward). `n_lin` = len(self.layers): num_hidden_layers+2,
# or 1 when num_hidden_layers == 0 (mlp.py:29-32). Dropout is identity at p=0.
# --------------------------------------------------------------------------------------


# Test instrumentation: when set, PRE_ACT_TAP(prefix, index, h) sees every pre-activation the ReLU
# MLPs below produce (tests/kinkfree.py conditions inputs away from ReLU kinks). No effect on values.
PRE_ACT_TAP = None


def _tap(pre, i, h):
    if PRE_ACT_TAP is not None:
        PRE_ACT_TAP(pre, i, h)
    return h


def mlp(p, pre, x, n_lin, ln=True, act=F.relu):
    for i in range(n_lin - 1):
        x = F.linear(x, p[f"{pre}.layers.{i}.weight"], p[f"{pre}.layers.{i}.bias"])
        x = act(_tap(pre, i, x))
    x = F.linear(x, p[f"{pre}.layers.{n_lin - 1}.weight"], p[f"{pre}.layers.{n_lin - 1}.bias"])
    if ln:
        w = p[f"{pre}.layer_norm.weight"]
        x = F.layer_norm(x, (w.shape[0],), w, p[f"{pre}.layer_norm.bias"], 1e-5)
    return x


def mlp_nlin(num_hidden_layers):
    return num_hidden_layers + 2 if num_hidden_layers > 0 else 1


# models/mgnLayer.py:93-105 (EdgeBlockSum.forward; Sequential ReLU,[Lin,ReLU]*n_hid,Lin,LN)
def edge_block_sum(p, pre, e, x, ei, n_hid):
    mlp_edge_attr = F.linear(e, p[f"{pre}.edge_lin"], None)
    mlp_src_feat = F.linear(x, p[f"{pre}.src_lin"], None)
    mlp_dst_feat = F.linear(x, p[f"{pre}.dst_lin"], p[f"{pre}.bias"])
    src, dst = ei.long()
    h = mlp_edge_attr + mlp_src_feat[src] + mlp_dst_feat[dst]
    h = F.relu(_tap(pre, 0, h))
    k = 1
    for _ in range(n_hid):
        h = F.relu(_tap(pre, k, F.linear(h, p[f"{pre}.mlp.{k}.weight"], p[f"{pre}.mlp.{k}.bias"])))
        k += 2
    h = F.linear(h, p[f"{pre}.mlp.{k}.weight"], p[f"{pre}.mlp.{k}.bias"])
    w = p.get(f"{pre}.mlp.{k + 1}.weight")
    if w is not None:
        h = F.layer_norm(h, (w.shape[0],), w, p[f"{pre}.mlp.{k + 1}.bias"], 1e-5)
    return h


# models/mgnLayer.py:32-49 (EdgeBlock.forward, do_concat_trick=False)
def edge_block_cat(p, pre, e, x, ei, n_hid, act=F.relu):
    row, col = ei
    h = torch.cat([e, x[row], x[col]], dim=-1)
    return mlp(p, f"{pre}.mlp", h, mlp_nlin(n_hid), ln=f"{pre}.mlp.layer_norm.weight" in p, act=act)


# models/mgnLayer.py:134-153 (NodeBlock.forward)
def node_block(p, pre, x, e, ei, n_hid, aggregation="add", act=F.relu):
    row, col = ei
    if aggregation == "mean":
        agg = scatter_mean(e, col, dim=0, dim_size=x.size(0))
    elif aggregation == "add":
        agg = scatter_add(e, col, dim=0, dim_size=x.size(0))
    else:
        raise ValueError(f"Unsupported aggregation method: {aggregation}")
    h = torch.cat([x, agg], dim=-1)
    return mlp(p, f"{pre}.mlp", h, mlp_nlin(n_hid), ln=f"{pre}.mlp.layer_norm.weight" in p, act=act)


# mlp.py:37: the MLPs' activation (getattr(F, activation_fn)); EdgeBlockSum's chain is always ReLU
# (mgnLayer.py:81)
def act_of(cfg):
    return getattr(F, cfg.get("activation_fn", "relu"))


# models/mgnLayer.py:177-213 (MeshGraphNetLayer.forward; memory-logging syncs omitted on CPU)
def gmp_layer(p, pre, x, e, ei, cfg):
    if cfg.get("do_concat_trick", False):
        e_new = edge_block_sum(p, f"{pre}.edge_block", e, x, ei, cfg["n_hid_edge"])
    else:
        e_new = edge_block_cat(p, f"{pre}.edge_block", e, x, ei, cfg["n_hid_edge"], act=act_of(cfg))
    e = e + e_new
    x_new = node_block(p, f"{pre}.node_block", x, e, ei, cfg["n_hid_node"], cfg.get("aggregation", "add"),
                       act=act_of(cfg))
    x = x + x_new
    return x, e


# models/mgn.py:108-139
def mgn_forward(p, x, ea, ei, cfg):
    xh = mlp(p, "node_encoder", x, mlp_nlin(cfg["n_hid_node_enc"]), act=act_of(cfg))
    eh = mlp(p, "edge_encoder", ea, mlp_nlin(cfg["n_hid_edge_enc"]), act=act_of(cfg))
    for l in range(cfg["processor_size"]):
        xh, eh = gmp_layer(p, f"layers.{l}", xh, eh, ei, cfg)
    return mlp(p, "decoder", xh, mlp_nlin(cfg["n_hid_dec"]), ln=False, act=act_of(cfg))


# models/bsms_mgn.py:217-301 (_downsample). `stable` selects the build's documented tie rule
# (stable (x, node id)); with tie-free x both orders agree.
def downsample(node, edge, ei, batch, pos, stride, stable=False):
    device = node.device
    num_nodes = node.size(0)
    f2c = torch.empty(num_nodes, dtype=torch.long, device=device)
    chunks = []
    uniq = torch.unique_consecutive(batch)
    off = 0
    for g in uniq.tolist():
        idx = torch.nonzero(batch == g, as_tuple=False).view(-1)
        if idx.numel() == 0:
            continue
        if pos is not None:
            gp = pos[idx]
            sidx = idx[torch.argsort(gp[:, 0], stable=stable)]
        else:
            sidx = idx
        cnt = sidx.numel()
        cl = torch.arange(cnt, device=device) // stride
        nc = int(cl[-1].item() + 1)
        f2c[sidx] = cl + off
        chunks.append(torch.full((nc,), g, device=device, dtype=torch.long))
        off += nc
    cbatch = torch.cat(chunks, 0) if chunks else torch.empty((0,), dtype=torch.long, device=device)
    Nc = cbatch.size(0)
    cnode = scatter_mean(node, f2c, dim=0, dim_size=Nc)
    cpos = scatter_mean(pos, f2c, dim=0, dim_size=Nc) if pos is not None else None
    row, col = ei
    keys = f2c[row] * max(Nc, 1) + f2c[col]
    ukeys, inv = torch.unique(keys, return_inverse=True)
    if ukeys.numel() > 0:
        cedge = scatter_mean(edge, inv, dim=0)
        cei = torch.stack([ukeys // max(Nc, 1), ukeys % max(Nc, 1)], 0)
    else:
        fd = edge.size(1) if edge.dim() > 1 else 1
        cedge = edge.new_zeros((0, fd))
        cei = ei.new_zeros((2, 0))
    return cnode, cedge, cei, cbatch, cpos, f2c


# models/bsms_mgn.py:126-215 (forward) with the layer schedule of :68-81
def bsms_schedule(processor_size, num_scales, layers_per_scale):
    if isinstance(layers_per_scale, int):
        down = [layers_per_scale] * max(num_scales - 1, 0)
    else:
        down = list(layers_per_scale)
    return down, max(1, processor_size - 2 * sum(down)), list(reversed(down))


def bsms_forward(p, x, ea, ei, cfg, batch=None, pos=None, stable=False):
    if batch is None:
        batch = x.new_zeros(x.size(0), dtype=torch.long)
    nh = mlp(p, "node_encoder", x, mlp_nlin(cfg["n_hid_node_enc"]), act=act_of(cfg))
    eh = mlp(p, "edge_encoder", ea, mlp_nlin(cfg["n_hid_edge_enc"]), act=act_of(cfg))
    down, bott, up = bsms_schedule(cfg["processor_size"], cfg["num_scales"], cfg["layers_per_scale"])
    assigns, skips = [], []
    cb, cp, cei, ce, cn = batch, pos, ei, eh, nh
    for s, cnt in enumerate(down):
        for l in range(cnt):
            cn, ce = gmp_layer(p, f"down_layers.{s}.{l}", cn, ce, cei, cfg)
        skips.append((cn, ce, cei, cb, cp))
        cn, ce, cei, cb, cp, a = downsample(cn, ce, cei, cb, cp, cfg["stride"], stable)
        assigns.append(a)
    for l in range(bott):
        cn, ce = gmp_layer(p, f"bottleneck_layers.{l}", cn, ce, cei, cfg)
    for s, cnt in enumerate(up):
        a = assigns[-(s + 1)] if assigns else None
        if a is not None:
            sn, se, sei, sb, sp = skips[-(s + 1)]
            cn = cn[a]
            cn = cn + sn
            ce, cei, cb, cp = se, sei, sb, sp
        for l in range(cnt):
            cn, ce = gmp_layer(p, f"up_layers.{s}.{l}", cn, ce, cei, cfg)
    return mlp(p, "decoder", cn, mlp_nlin(cfg["n_hid_dec"]), ln=False, act=act_of(cfg))


# torch_geometric.nn.global_{add,mean,max}_pool (PyG; unpinned, not installed): size = batch.max()+1,
# scatter 'sum' / 'mean' (count clamped to 1) / 'max' (zero-initialised amax, include_self=False)
def global_pool(x, batch, method):
    size = int(batch.max()) + 1
    idx = batch.view(-1, 1).expand_as(x)
    out = x.new_zeros(size, x.size(1))
    if method == "max":
        return out.scatter_reduce_(0, idx, x, reduce="amax", include_self=False)
    out = out.scatter_add_(0, idx, x)
    if method == "mean":
        cnt = x.new_zeros(size).scatter_add_(0, batch, x.new_ones(x.size(0))).clamp_(min=1)
        out = out / cnt.view(-1, 1)
    return out


# models/poolmgn.py:120-158 (poolMGN.forward)
def poolmgn_forward(p, x, ea, ei, cfg, batch=None):
    g = mlp(p, "global_encoder", x, mlp_nlin(cfg["n_hid_global_enc"]), ln=False, act=act_of(cfg))
    if batch is not None:
        g = global_pool(g, batch, cfg["global_pool_method"])
        g = g.repeat_interleave(torch.bincount(batch), dim=0)
    else:
        g = global_pool(g, torch.zeros(x.size(0), dtype=torch.long), cfg["global_pool_method"])
        g = g.repeat(x.size(0), 1)
    xh = mlp(p, "node_encoder", torch.cat((x, g), dim=-1), mlp_nlin(cfg["n_hid_node_enc"]), act=act_of(cfg))
    eh = mlp(p, "edge_encoder", ea, mlp_nlin(cfg["n_hid_edge_enc"]), act=act_of(cfg))
    for l in range(cfg["processor_size"]):
        xh, eh = gmp_layer(p, f"layers.{l}", xh, eh, ei, cfg)
    return mlp(p, "decoder", xh, mlp_nlin(cfg["n_hid_dec"]), ln=False, act=act_of(cfg))


def cfg_from_kwargs(**kw):
    """Map BiStridedMeshGraphNet / MeshGraphNet ctor kwargs (reference names) to oracle cfg."""
    return dict(
        processor_size=kw.get("processor_size", 15),
        n_hid_node=kw.get("num_hidden_layers_node_processor", 1),
        n_hid_edge=kw.get("num_hidden_layers_edge_processor", 1),
        n_hid_node_enc=kw.get("num_hidden_layers_node_encoder", 1),
        n_hid_edge_enc=kw.get("num_hidden_layers_edge_encoder", 1),
        n_hid_dec=kw.get("num_hidden_layers_decoder", 1),
        aggregation=kw.get("aggregation", "add"),
        do_concat_trick=kw.get("do_concat_trick", False),
        num_scales=kw.get("num_scales", 3),
        layers_per_scale=kw.get("layers_per_scale", 2),
        stride=kw.get("stride", 2),
        global_pool_method=kw.get("global_pool_method", "mean"),
        n_hid_global_enc=kw.get("num_hidden_layers_global_encoder", 1),
        activation_fn=kw.get("activation_fn", "relu"),
    )


# dataset.py:39-64 (compute_edge_attr)
def compute_edge_attr(pos, edge_index):
    source_pos = pos[edge_index[0]]
    target_pos = pos[edge_index[1]]
    edge_vec = target_pos - source_pos
    edge_length = torch.norm(edge_vec, dim=1, keepdim=True)
    return torch.cat([edge_vec, edge_length], dim=1)


# dataset.py:358-392 (compute_normalization_stats)
def compute_normalization_stats(xs, eas, ys):
    x_std, x_mean = torch.std_mean(torch.vstack(xs), dim=0)
    e_std, e_mean = torch.std_mean(torch.vstack(eas), dim=0)
    y_std, y_mean = torch.std_mean(torch.vstack(ys), dim=0)
    eps = 1e-8
    return {"node_mean": x_mean, "node_std": torch.clamp(x_std, min=eps), "edge_mean": e_mean,
            "edge_std": torch.clamp(e_std, min=eps), "target_mean": y_mean, "target_std": torch.clamp(y_std, min=eps)}


# dataset.py:394-409 (normalize_data, one tensor)
def normalize(v, mean, std):
    return (v - mean) / std
