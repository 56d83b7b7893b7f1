"""Device-side data preparation, mirroring the reference's dataset helpers:

  compute_edge_attr            dataset.py:39-64   [pos[dst] - pos[src], |.|] per edge
  compute_node_features        dataset.py:66-106  cat(pos, normals, broadcast global params)
  compute_normalization_stats  dataset.py:358-392 torch.std_mean over the stacked data, std >= 1e-8
  normalize_data               dataset.py:394-409 (v - mean) / std, in place on each sample
  denormalize_predictions      dataset.py:411-421 v * std + mean
  collate                      train.py:50-51     PyG Batch.from_data_list of mesh samples

Samples are any objects with tensor attributes (PyG `Data` or a plain namespace); every tensor
lives on the MI355X, and each op is one libaerognn pass (agn_edge_features, agn_normalize,
agn_col_stats, agn_collate). `compute_edge_attr(..., perm=level.perm)` writes the features
directly in a level's receiver-grouped (CSC) order, i.e. the edge encoder's input order.
"""
from __future__ import annotations

import ctypes as C
import types

import torch

from . import _lib as L
from ._lib import check, ptr
from .core import require_device, stream

EPS = 1e-8  # dataset.py:386


def _f32(t):
    return t if (t.dtype == torch.float32 and t.is_contiguous()) else t.float().contiguous()


def compute_edge_attr(data=None, *, pos=None, edge_index=None, perm=None, stats=None, dtype=None):
    """[E, pos_dim + 1] edge features (dataset.py:52-62); with `stats` normalised by
    (edge_mean, edge_std); with `perm` row i is edge perm[i]."""
    pos = data.pos if pos is None else pos
    edge_index = data.edge_index if edge_index is None else edge_index
    require_device(pos, edge_index, perm)
    p32 = _f32(pos)
    # the kernel reads int64 indices: other integer dtypes are converted (int32 levels included)
    ei = edge_index.long().contiguous()
    if perm is not None:
        perm = perm.long().contiguous()
    ne = ei.shape[1] if perm is None else perm.numel()
    out = torch.empty(ne, p32.shape[1] + 1, dtype=torch.float32, device=p32.device)
    mean = std = None
    if stats is not None:
        mean, std = _f32(stats["edge_mean"]), _f32(stats["edge_std"])
        require_device(mean, std)
        if mean.numel() != p32.shape[1] + 1 or std.numel() != p32.shape[1] + 1:
            raise ValueError("edge normalization stats must have pos_dim + 1 entries")
    check(L.lib().agn_edge_features(int(ne), int(ei.shape[1]), int(p32.shape[1]), ptr(ei), ptr(p32), p32.stride(0),
                                    ptr(perm), ptr(mean), ptr(std), ptr(out), stream()), "edge_features")
    return out if dtype is None else out.to(dtype)


def compute_node_features(data, var_keys=()):
    """cat(pos, normals (if present), per-sample global parameters broadcast to every node)
    (dataset.py:78-104)."""
    require_device(data.pos)
    feats = [data.pos]
    if getattr(data, "normals", None) is not None:
        feats.append(data.normals)
    n = data.pos.size(0)
    for key in var_keys:
        if hasattr(data, key):
            v = getattr(data, key)
            v = torch.as_tensor(v, dtype=data.pos.dtype, device=data.pos.device)
            v = v if v.dim() > 0 else v.unsqueeze(0)
            feats.append(v.to(data.pos.dtype).unsqueeze(0).expand(n, -1))
    return torch.cat(feats, dim=1)


def _col_stats(x):
    x = _f32(x)
    n, k = x.shape
    mean = torch.empty(k, dtype=torch.float32, device=x.device)
    std = torch.empty(k, dtype=torch.float32, device=x.device)
    scratch = torch.empty(int(L.lib().agn_col_stats_temp_bytes(n, k)), dtype=torch.uint8, device=x.device)
    check(L.lib().agn_col_stats(n, k, ptr(x), x.stride(0), ptr(mean), ptr(std), C.c_float(EPS), ptr(scratch), stream()),
          "col_stats")
    return mean, std


def compute_normalization_stats(data_list):
    """torch.std_mean over the stacked x / edge_attr / y of the samples (unbiased std, clamped to
    1e-8): the dict of dataset.py:376-392, fp32 device tensors."""
    xs = torch.cat([d.x for d in data_list])
    es = torch.cat([d.edge_attr for d in data_list])
    ys = torch.cat([d.y for d in data_list])
    require_device(xs, es, ys)
    st = {}
    st["node_mean"], st["node_std"] = _col_stats(xs)
    st["edge_mean"], st["edge_std"] = _col_stats(es)
    st["target_mean"], st["target_std"] = _col_stats(ys)
    return st


def _normalize(t, mean, std, inverse=False):
    require_device(t, mean, std)  # statistics are read by the kernel: device tensors only
    if mean.numel() != t.shape[1] or std.numel() != t.shape[1]:
        raise ValueError(f"normalization stats of size {mean.numel()}/{std.numel()} for {t.shape[1]} columns")
    t32 = _f32(t)
    out = torch.empty_like(t32)
    check(L.lib().agn_normalize(t32.shape[0], t32.shape[1], ptr(t32), t32.stride(0), ptr(_f32(mean)), ptr(_f32(std)),
                                ptr(out), out.stride(0), int(inverse), stream()), "normalize")
    return out if t.dtype == torch.float32 else out.to(t.dtype)


def normalize_data(data_list, stats):
    """x, edge_attr and y of every sample <- (v - mean) / std (dataset.py:401-409)."""
    for d in data_list:
        d.x = _normalize(d.x, stats["node_mean"], stats["node_std"])
        d.edge_attr = _normalize(d.edge_attr, stats["edge_mean"], stats["edge_std"])
        d.y = _normalize(d.y, stats["target_mean"], stats["target_std"])


def denormalize_predictions(predictions, stats):
    """predictions * target_std + target_mean (dataset.py:411-421)."""
    return _normalize(predictions, stats["target_mean"], stats["target_std"], inverse=True)


def collate(data_list, keys=("x", "edge_attr", "y", "pos")):
    """PyG Batch.from_data_list for mesh samples: rows of `keys` concatenated, edge_index offset
    by each mesh's first node id, `batch` = mesh index per node (agn_collate, one pass)."""
    dev = data_list[0].edge_index.device
    out = types.SimpleNamespace()
    for k in keys:
        vals = [getattr(d, k, None) for d in data_list]
        if all(v is not None for v in vals):
            setattr(out, k, torch.cat(vals, 0))
    nn = [int(d.num_nodes) if getattr(d, "num_nodes", None) is not None else int(d.x.shape[0]) for d in data_list]
    ne = [int(d.edge_index.shape[1]) for d in data_list]
    node_off = torch.tensor([0] + nn, dtype=torch.int64).cumsum(0).to(dev)
    edge_off = torch.tensor([0] + ne, dtype=torch.int64).cumsum(0).to(dev)
    ei = torch.cat([d.edge_index.long() for d in data_list], 1).contiguous()  # agn_collate: int64, in place
    require_device(ei)
    batch = torch.empty(sum(nn), dtype=torch.int64, device=dev)
    check(L.lib().agn_collate(len(data_list), int(sum(ne)), int(sum(nn)), ptr(edge_off), ptr(node_off), ptr(ei),
                              ptr(batch), stream()), "collate")
    out.edge_index, out.batch, out.num_nodes, out.num_graphs = ei, batch, sum(nn), len(data_list)
    return out
