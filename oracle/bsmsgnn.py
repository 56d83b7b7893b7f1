"""CPU oracle for the stale BSMS-GNN operators — TEST INFRASTRUCTURE ONLY.

Restates the design that survives only as CPython-3.11 bytecode in the reference
(`models/__pycache__/bistride_ops.cpython-311.pyc`, the old `bsms_mgn.cpython-311.pyc`),
following the semantics recovered in SURVEY.md Appendix A (no reference execution is possible:
the bytecode cannot be loaded by this interpreter). PARITY UNPINNED: no golden vector of the
reference exists for these ops; this restatement is the checker, and its own tests pin it to
hand-computed cases (tests/test_bsmsgnn_cpu.py).

Only tests/ may import this module; the product path (aero-gnn_amd) never does.
Citations: "bo@L" = bistride_ops.pyc source line L, "bm@L" = old bsms_mgn.pyc source line L.
"""
from collections import deque

import torch
import torch.nn.functional as F

from .refcpu import mlp, mlp_nlin, scatter_add, scatter_mean


# bo@21 BistridePooling.bfs_distance
def bfs_distance(edge_index, num_nodes, start_node):
    dist = torch.full((num_nodes,), -1, dtype=torch.long)
    dist[start_node] = 0
    adj = [[] for _ in range(num_nodes)]
    src, dst = edge_index[0].tolist(), edge_index[1].tolist()
    for s, d in zip(src, dst):
        adj[s].append(d)
    q = deque([start_node])
    while q:
        u = q.popleft()
        cur = int(dist[u])
        for v in adj[u]:
            if dist[v] == -1:
                dist[v] = cur + 1
                q.append(v)
    return dist


# bo@56 BistridePooling.select_bistride_nodes
def select_seed(edge_index, num_nodes, pos=None):
    if pos is not None:
        center = pos.mean(dim=0)
        return int(torch.argmin(torch.norm(pos - center, dim=1)).item())
    deg = torch.bincount(edge_index[0], minlength=num_nodes)
    return int(torch.argmax(deg).item())


def select_bistride_nodes(edge_index, num_nodes, pos=None, seed=None):
    """`seed` overrides the seed rule (tests pin the GPU's seed choice separately)."""
    if seed is None:
        seed = select_seed(edge_index, num_nodes, pos)
    d = bfs_distance(edge_index, num_nodes, seed)
    sel = torch.where((d % 2 == 0) & (d >= 0))[0]
    if len(sel) < num_nodes * 0.3:
        sel = torch.where(d >= 0)[0]
    return sel


# bm@32 MultiScaleGraphPreprocessor.create_multiscale_graph
def create_multiscale_graph(edge_index, pos, num_nodes, num_levels, seeds=None):
    multi = {"edge_indices": [edge_index], "node_indices": [], "num_nodes": [num_nodes], "positions": [pos]}
    ei, cp, n = edge_index, pos, num_nodes
    for lvl in range(num_levels):
        sel = select_bistride_nodes(ei, n, cp, None if seeds is None else seeds[lvl])
        imap = torch.full((n,), -1, dtype=torch.long)
        imap[sel] = torch.arange(len(sel))
        src, dst = ei
        mask = (imap[src] >= 0) & (imap[dst] >= 0)
        ns, nd = imap[src[mask]], imap[dst[mask]]
        keep = ns != nd
        ei = torch.stack([ns[keep], nd[keep]], 0)
        cp = cp[sel] if cp is not None else None
        n = len(sel)
        multi["edge_indices"].append(ei)
        multi["node_indices"].append(sel)
        multi["num_nodes"].append(n)
        multi["positions"].append(cp)
    return multi


# bo@102 Unpool.forward
def unpool(x_coarse, indices, num_nodes_fine):
    out = x_coarse.new_zeros((num_nodes_fine, x_coarse.shape[1]))
    out[indices] = x_coarse
    return out


# bo@152 WeightedEdgeConv.compute_edge_weights
def wec_weights(p, pre, x, edge_index, pos):
    src, dst = edge_index
    el = torch.norm(pos[dst] - pos[src], dim=1, keepdim=True)
    feat = torch.cat([x[src], x[dst], el.to(x.dtype)], dim=1)
    h = F.relu(F.linear(feat, p[f"{pre}.edge_weight_mlp.0.weight"], p[f"{pre}.edge_weight_mlp.0.bias"]))
    return torch.sigmoid(F.linear(h, p[f"{pre}.edge_weight_mlp.2.weight"], p[f"{pre}.edge_weight_mlp.2.bias"]))


# bo@173 WeightedEdgeConv.forward
def wec_forward(p, pre, x, edge_index, pos, edge_weights=None, compute_weights=True, aggr="add"):
    if compute_weights and edge_weights is None:
        edge_weights = wec_weights(p, pre, x, edge_index, pos)
    src, dst = edge_index
    xt = F.linear(x, p[f"{pre}.transform.weight"], p[f"{pre}.transform.bias"])
    m = xt[src] * edge_weights
    if aggr == "add":
        out = scatter_add(m, dst, dim=0, dim_size=x.shape[0])
    elif aggr == "mean":
        out = scatter_mean(m, dst, dim=0, dim_size=x.shape[0])
    else:
        raise ValueError(f"Unknown aggregation: {aggr}")
    return out, edge_weights


def _seq(p, pre, x):
    """Sequential(Linear, ReLU, Linear, LayerNorm) of GMP (bo@216)."""
    h = F.relu(F.linear(x, p[f"{pre}.0.weight"], p[f"{pre}.0.bias"]))
    h = F.linear(h, p[f"{pre}.2.weight"], p[f"{pre}.2.bias"])
    return F.layer_norm(h, (h.shape[-1],), p[f"{pre}.3.weight"], p[f"{pre}.3.bias"])


# bo@235 GMP.forward
def gmp(p, pre, x, edge_attr, edge_index):
    src, dst = edge_index
    e = edge_attr + _seq(p, f"{pre}.edge_mlp", torch.cat([x[src], x[dst], edge_attr], dim=1))
    agg = scatter_add(e, dst, dim=0, dim_size=x.size(0))
    x = x + _seq(p, f"{pre}.node_mlp", torch.cat([x, agg], dim=1))
    return x, e


# bm@145 BSMSGMP.forward
def bsmsgmp(p, pre, x, edge_attrs, edge_indices, node_indices, num_nodes_list, positions, num_levels):
    edge_attrs = list(edge_attrs)
    skips, ws = [], []
    for i in range(num_levels):
        x, edge_attrs[i] = gmp(p, f"{pre}.down_gmps.{i}", x, edge_attrs[i], edge_indices[i])
        skips.append(x.clone())
        xc, w = wec_forward(p, f"{pre}.down_edge_convs.{i}", x, edge_indices[i], positions[i], compute_weights=True)
        ws.append(w)
        x = x + xc
        x = x[node_indices[i]]
    x, edge_attrs[-1] = gmp(p, f"{pre}.bottom_gmp", x, edge_attrs[-1], edge_indices[-1])
    for i in range(num_levels - 1, -1, -1):
        x = unpool(x, node_indices[i], num_nodes_list[i])
        xc, _ = wec_forward(p, f"{pre}.up_edge_convs.{i}", x, edge_indices[i], positions[i],
                            edge_weights=ws[i], compute_weights=False)
        x = x + xc + skips[i]
    return x


# bm@281 BSMS_MeshGraphNet.forward
def bsms_gnn_forward(p, node_attr, edge_attr, multi, num_levels, n_hid_enc=2, n_hid_dec=2):
    nh = mlp(p, "node_encoder", node_attr, mlp_nlin(n_hid_enc))
    eh = mlp(p, "edge_encoder", edge_attr, mlp_nlin(n_hid_enc))
    eas = [eh] + [nh.new_zeros((ei.shape[1], nh.shape[1])) for ei in multi["edge_indices"][1:]]
    x = bsmsgmp(p, "bsgmp", nh, eas, multi["edge_indices"], multi["node_indices"], multi["num_nodes"],
                multi["positions"], num_levels)
    return mlp(p, "decoder", x, mlp_nlin(n_hid_dec), ln=False)
