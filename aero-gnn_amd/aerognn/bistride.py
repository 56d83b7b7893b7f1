"""Device-side bi-stride graph coarsening of the stale BSMS-GNN design:
BistridePooling.bfs_distance / select_bistride_nodes (bistride_ops.pyc @21, @56) and
MultiScaleGraphPreprocessor.create_multiscale_graph (old bsms_mgn.pyc @32).

All integer work runs in libaerognn (level-synchronous BFS, seed reductions, order-preserving
compactions). The results are exact: BFS distances do not depend on visiting order, and the
selections / sub-graphs keep ascending node ids and the caller's edge order.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L
from ._lib import check, ptr
from .core import stream
from .graph import group_by

I32 = torch.int32
I64 = torch.int64


def out_adjacency(edge_index: torch.Tensor, num_nodes: int):
    """CSR of edge_index[0] -> edge_index[1] (rowptr int32 [n+1], neighbours int32 [E])."""
    perm, rowptr = group_by(edge_index[0].to(I32), num_nodes)
    nbr = edge_index[1].index_select(0, perm.long()).to(I32)
    return rowptr, nbr


def bfs_distance(edge_index: torch.Tensor, num_nodes: int, start_node: int, adj=None) -> torch.Tensor:
    """Hop distances from `start_node` over out-edges; -1 = unreachable (int64, on device)."""
    dev = edge_index.device
    rowptr, nbr = adj if adj is not None else out_adjacency(edge_index, num_nodes)
    dist = torch.empty(num_nodes, dtype=I32, device=dev)
    work = torch.empty(int(L.lib().agn_bfs_work_ints(num_nodes)), dtype=I32, device=dev)
    levels = C.c_int(0)
    check(L.lib().agn_bfs_distance(ptr(rowptr), ptr(nbr), num_nodes, int(start_node), ptr(dist), ptr(work),
                                   C.byref(levels), stream()), "bfs_distance")
    return dist.long()


def bistride_seed(edge_index, num_nodes, pos=None, adj=None) -> int:
    """argmin |pos - mean(pos)| when pos is given, else argmax out-degree (first index on ties)."""
    dev = edge_index.device
    seed = torch.empty(1, dtype=I32, device=dev)
    if pos is not None:
        p = pos.float().contiguous()
        check(L.lib().agn_center_seed(ptr(p), num_nodes, p.shape[1], p.stride(0), ptr(seed), stream()), "seed")
    else:
        rowptr = adj[0] if adj is not None else out_adjacency(edge_index, num_nodes)[0]
        check(L.lib().agn_maxdeg_seed(ptr(rowptr), num_nodes, ptr(seed), stream()), "seed")
    return int(seed.item())


def select_from_distance(dist: torch.Tensor, num_nodes: int) -> torch.Tensor:
    dev = dist.device
    d32 = dist.to(I32).contiguous()
    sel = torch.empty(max(num_nodes, 1), dtype=I32, device=dev)
    work = torch.empty(int(L.lib().agn_compact_work_ints(num_nodes)), dtype=I32, device=dev)
    n = C.c_int(0)
    check(L.lib().agn_bistride_select(ptr(d32), num_nodes, ptr(sel), C.byref(n), ptr(work), stream()), "select")
    return sel[:n.value].long()


def select_bistride_nodes(edge_index, num_nodes, pos=None, seed=None) -> torch.Tensor:
    """bistride_ops @56: nodes at even BFS depth from the seed (all reachable if < 30 %)."""
    if num_nodes == 0:
        return torch.empty(0, dtype=I64, device=edge_index.device)
    adj = out_adjacency(edge_index, num_nodes)
    if seed is None:
        seed = bistride_seed(edge_index, num_nodes, pos, adj)
    dist = bfs_distance(edge_index, num_nodes, seed, adj)
    return select_from_distance(dist, num_nodes)


def subgraph_edges(edge_index: torch.Tensor, sel: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """Edges with both ends selected, remapped to coarse ids, self loops dropped (order kept)."""
    dev = edge_index.device
    E = edge_index.shape[1]
    lib = L.lib()
    sel32 = sel.to(I32).contiguous()
    imap = torch.empty(max(num_nodes, 1), dtype=I32, device=dev)
    check(lib.agn_index_map(ptr(sel32), sel32.numel(), num_nodes, ptr(imap), stream()), "index_map")
    ei = edge_index.to(I64).contiguous()
    osrc = torch.empty(max(E, 1), dtype=I64, device=dev)
    odst = torch.empty(max(E, 1), dtype=I64, device=dev)
    work = torch.empty(int(lib.agn_compact_work_ints(E)), dtype=I32, device=dev)
    n = C.c_int(0)
    check(lib.agn_subgraph_edges(ptr(ei[0]), ptr(ei[1]), E, ptr(imap), ptr(osrc), ptr(odst), C.byref(n), ptr(work),
                                 stream()), "subgraph_edges")
    return torch.stack([osrc[:n.value], odst[:n.value]], 0)


def create_multiscale_graph(edge_index, pos, num_nodes, num_levels):
    """old bsms_mgn @32: {'edge_indices', 'node_indices', 'num_nodes', 'positions'} lists."""
    multi = {"edge_indices": [edge_index], "node_indices": [], "num_nodes": [num_nodes], "positions": [pos]}
    ei, cp, n = edge_index, pos, num_nodes
    for _ in range(num_levels):
        sel = select_bistride_nodes(ei, n, cp)
        ei = subgraph_edges(ei, sel, n)
        cp = cp.index_select(0, sel) if cp is not None else None
        n = int(sel.numel())
        multi["edge_indices"].append(ei)
        multi["node_indices"].append(sel)
        multi["num_nodes"].append(n)
        multi["positions"].append(cp)
    return multi
