"""Bistride operations of the BSMS-GNN design — drop-in for the reference's stale
`models/bistride_ops` (CPython-3.11 bytecode only, no .py; semantics recovered in SURVEY
Appendix A, "bo@L" = source line L of that module). Based on BSMS-GNN (Cao et al., ICML 2023).

Every op runs on libaerognn (MI355X): BFS and the bi-stride selection as device integer
kernels, Unpool as a row scatter, WeightedEdgeConv as a fused per-receiver kernel, GMP on the
fused MLP kernels. There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

import torch
from torch import nn

from aerognn import bistride as B
from aerognn.core import require_device
from aerognn.functions import GMPFn, LayerSpec, UnpoolRowsFn, WECFn, WECGivenFn, WecSpec, from_csc, to_csc
from aerognn.graph import Level

__all__ = ["BistridePooling", "Unpool", "WeightedEdgeConv", "GMP"]


class BistridePooling:
    """Selects the nodes on every other BFS frontier (bo@13)."""

    @staticmethod
    def bfs_distance(edge_index, num_nodes, start_node):
        """bo@21: hop distances from start_node over edge_index[0] -> [1]; -1 if unreachable."""
        require_device(edge_index)
        return B.bfs_distance(edge_index, int(num_nodes), int(start_node))

    @staticmethod
    def select_bistride_nodes(edge_index, num_nodes, pos=None):
        """bo@56: seed = argmin |pos - mean(pos)| (or max out-degree without pos); keep even BFS
        depths, or every reachable node if that keeps fewer than 30 %. Ascending int64 ids."""
        require_device(edge_index, pos)
        return B.select_bistride_nodes(edge_index, int(num_nodes), pos)


class Unpool(nn.Module):
    """bo@102: x_fine = zeros(N_fine, C); x_fine[indices] = x_coarse (2-D or batched 3-D)."""

    def __init__(self):
        super().__init__()

    def forward(self, x_coarse, indices, num_nodes_fine):
        require_device(x_coarse, indices)
        idx = indices.to(torch.int32).contiguous()
        if x_coarse.dim() == 2:
            return UnpoolRowsFn.apply(x_coarse, idx, int(num_nodes_fine))
        b, nc, c = x_coarse.shape
        rows = x_coarse.transpose(0, 1).reshape(nc, b * c)
        out = UnpoolRowsFn.apply(rows, idx, int(num_nodes_fine))
        return out.view(int(num_nodes_fine), b, c).transpose(0, 1)


def _level_of(edge_index, n, cache=None):
    key = (edge_index.data_ptr(), tuple(edge_index.shape), n)
    if cache is not None and key in cache:
        return cache[key]
    lv = Level.from_edge_index(edge_index, n)
    if cache is not None:
        cache[key] = lv
    return lv


class WeightedEdgeConv(nn.Module):
    """bo@131-210: edge weights w = MLP(cat[x_src, x_dst, |pos_dst - pos_src|]) in (0, 1),
    out = scatter_{add|mean}(transform(x)[src] * w, dst). Returns (out, edge_weights [E, 1])."""

    def __init__(self, in_dim, out_dim, aggr='add'):
        super().__init__()
        self.in_dim, self.out_dim, self.aggr = in_dim, out_dim, aggr
        self.edge_weight_mlp = nn.Sequential(nn.Linear(2 * in_dim + 1, 64), nn.ReLU(), nn.Linear(64, 1), nn.Sigmoid())
        self.transform = nn.Linear(in_dim, out_dim)
        self._spec = None

    def spec(self):
        if self._spec is None:
            self._spec = WecSpec(self)
        return self._spec

    def _mean(self):
        if self.aggr == 'add':
            return False
        if self.aggr == 'mean':
            return True
        raise ValueError(f"Unknown aggregation: {self.aggr}")

    def compute_edge_weights(self, x, edge_index, pos, level=None):
        """bo@152: [E, 1] weights in the caller's edge order."""
        return self.forward(x, edge_index, pos, level=level)[1]

    def forward(self, x, edge_index, pos, edge_weights=None, compute_weights=True, level=None):
        require_device(x, edge_index, pos, edge_weights)
        mean = self._mean()
        lv = level if level is not None else _level_of(edge_index, x.shape[0])
        s = self.spec()
        if compute_weights and edge_weights is None:
            out, w = WECFn.apply(x, pos, lv, s, mean, *s.params())
            return out, w
        if edge_weights is None:
            raise ValueError("WeightedEdgeConv: compute_weights=False needs edge_weights")
        out = WECGivenFn.apply(x, edge_weights, lv, s, mean, self.transform.weight, self.transform.bias)
        return out, edge_weights


class GMP(nn.Module):
    """bo@216-250: e' = e + LN(Lin(act(Lin(cat[x_src, x_dst, e])))), x' = x + LN(Lin(act(Lin(cat[x, sum_dst e']))))."""

    def __init__(self, node_dim, edge_dim, hidden_dim, activation='relu'):
        super().__init__()
        act = nn.ReLU() if activation == 'relu' else nn.SiLU()
        self.edge_mlp = nn.Sequential(nn.Linear(2 * node_dim + edge_dim, hidden_dim), act,
                                      nn.Linear(hidden_dim, edge_dim), nn.LayerNorm(edge_dim))
        self.node_mlp = nn.Sequential(nn.Linear(node_dim + edge_dim, hidden_dim), act,
                                      nn.Linear(hidden_dim, node_dim), nn.LayerNorm(node_dim))
        self._spec = None

    def spec(self):
        if self._spec is None:
            self._spec = LayerSpec.from_gmp(self)
        return self._spec

    def forward(self, x, edge_attr, edge_index, level=None):
        """Edges in the caller's order in and out (the level's CSC order internally)."""
        require_device(x, edge_attr, edge_index)
        lv = level if level is not None else _level_of(edge_index, x.shape[0])
        xo, eo = self.forward_level(x, to_csc(edge_attr, lv), lv)
        return xo, from_csc(eo, lv)

    def forward_level(self, x, edge_attr_csc, level):
        s = self.spec()
        s.pack.update(x.dtype, x.device)
        return GMPFn.apply(x, edge_attr_csc, level, s, torch.is_grad_enabled(), *s.params())
