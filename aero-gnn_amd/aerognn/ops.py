"""torch.ops.aerognn.* — libaerognn's row-grouping kernels as registered PyTorch operators
(VERDICT r1 item 9).

The reference reaches these operations through third-party Python ops: torch_scatter's
scatter_add / scatter_mean / scatter_max along dim 0 (mgnLayer.py:144,146, bsms_mgn.py:265,270,
283) and torch_geometric's global pools (poolmgn.py:132-141). Registered here with
torch.library, they have a schema, fake (meta) kernels for shape propagation under
torch.compile / FakeTensorMode, and autograd formulas that are themselves torch.ops.aerognn ops:

  scatter_sum(src [n,k], index [n], dim_size, mean=False) -> [dim_size, k]
      out[r] = sum (or mean) of src[i] over index[i] == r, in increasing i (torch_scatter's CPU
      order; empty groups give 0). Grouping: agn_radix_sort_u64 + agn_row_ptr; sum:
      agn_segment_sum. Backward: gather_rows (mean: divided by the group size).
  group_ptr(index [n], dim_size) -> int32 [dim_size + 1] group offsets (radix sort + agn_row_ptr).
  gather_rows(src [m,k], index [n], rowptr=None) -> [n, k]
      out[i] = src[index[i]] (/ group size of index[i] when rowptr is given): agn_gather_rows.
      Backward: scatter_sum.
  scatter_max(src [n,k], index [n], dim_size) -> (out [dim_size,k], argmax [dim_size,k] int64)
      per column maximum and the first row attaining it (NaN wins, as in torch's max); empty
      groups give 0 and argmax = n (torch_scatter's convention): agn_segment_max. Backward:
      agn_segment_max_backward (gradient to the argmax row only).
  edge_features(pos [N,d], edge_index [2,E], mean=None, std=None) -> [E, d+1]
      [pos[dst] - pos[src], |.|] (dataset.py:52-62), optionally normalised: agn_edge_features.

The fused MLP / MeshGraphNet-layer kernels are not registered as operators: their calls carry
packed-weight caches and a per-level CSC plan (Python objects), so they stay
torch.autograd.Functions behind the reference's nn.Module API (models/).

Every op requires device tensors and raises on CPU inputs: there is no CPU fallback.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor

from .core import gather_rows as _gather_rows
from .core import require_device, segment_max as _segment_max
from .core import segment_max_backward as _segment_max_backward
from .core import segment_sum as _segment_sum

I32 = torch.int32


def _groups(index: Tensor, dim_size: int):
    from .graph import group_by
    idx = index.to(I32)
    if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= dim_size):
        raise IndexError(f"scatter index out of range [0, {dim_size})")
    return group_by(idx, dim_size)


def _rows2d(t: Tensor, what: str) -> Tensor:
    if t.dim() != 2:
        raise ValueError(f"{what}: expected a 2-D [rows, features] tensor, got shape {tuple(t.shape)}")
    return t.contiguous()


# ------------------------------------------------------------------------------- group_ptr
@torch.library.custom_op("aerognn::group_ptr", mutates_args=())
def group_ptr(index: Tensor, dim_size: int) -> Tensor:
    """int32 [dim_size + 1] offsets of the groups of `index` (group sizes = diff): the count a
    mean divides by, as a tensor op so autograd formulas stay traceable."""
    require_device(index)
    return _groups(index, dim_size)[1]


@group_ptr.register_fake
def _(index, dim_size):
    return index.new_empty(dim_size + 1, dtype=I32)


# ------------------------------------------------------------------------------- scatter_sum
@torch.library.custom_op("aerognn::scatter_sum", mutates_args=())
def scatter_sum(src: Tensor, index: Tensor, dim_size: int, mean: bool = False) -> Tensor:
    require_device(src, index)
    src = _rows2d(src, "scatter_sum")
    if index.numel() != src.shape[0]:
        raise ValueError("scatter_sum: index must have one entry per row of src")
    perm, rowptr = _groups(index, dim_size)
    out = torch.empty(dim_size, src.shape[1], dtype=src.dtype, device=src.device)
    if dim_size:
        _segment_sum(dim_size, src.shape[1], rowptr, perm, src, out, mean=mean)
    return out


@scatter_sum.register_fake
def _(src, index, dim_size, mean=False):
    return src.new_empty(dim_size, src.shape[1])


def _scatter_sum_ctx(ctx, inputs, output):
    src, index, dim_size, mean = inputs
    ctx.save_for_backward(index)
    ctx.mean = mean
    ctx.dim_size = dim_size


def _scatter_sum_bwd(ctx, g):
    (index,) = ctx.saved_tensors
    rowptr = torch.ops.aerognn.group_ptr(index, ctx.dim_size) if ctx.mean else None
    return torch.ops.aerognn.gather_rows(g, index, rowptr), None, None, None


torch.library.register_autograd("aerognn::scatter_sum", _scatter_sum_bwd, setup_context=_scatter_sum_ctx)


# ------------------------------------------------------------------------------- gather_rows
@torch.library.custom_op("aerognn::gather_rows", mutates_args=())
def gather_rows(src: Tensor, index: Tensor, rowptr: Optional[Tensor] = None) -> Tensor:
    require_device(src, index, rowptr)
    src = _rows2d(src, "gather_rows")
    idx = index.to(I32).contiguous()
    if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= src.shape[0]):
        raise IndexError(f"gather index out of range [0, {src.shape[0]})")
    out = torch.empty(idx.numel(), src.shape[1], dtype=src.dtype, device=src.device)
    if idx.numel():
        _gather_rows(idx.numel(), src.shape[1], idx, src, out,
                     cnt_ptr=rowptr.to(I32).contiguous() if rowptr is not None else None)
    return out


@gather_rows.register_fake
def _(src, index, rowptr=None):
    return src.new_empty(index.numel(), src.shape[1])


def _gather_ctx(ctx, inputs, output):
    src, index, rowptr = inputs
    ctx.save_for_backward(index, rowptr)
    ctx.n = src.shape[0]


def _gather_bwd(ctx, g):
    index, rowptr = ctx.saved_tensors
    # d src[r] = sum over i with index[i] == r of g[i], divided by the caller's group size
    # max(rowptr[r+1] - rowptr[r], 1) when the forward divided by it (any rowptr, not only
    # group_ptr(index))
    if rowptr is None:
        return torch.ops.aerognn.scatter_sum(g, index, ctx.n, False), None, None
    # sum and divide in fp32 and round once, as the forward's in-kernel fp32 division does (a bf16
    # count would round group sizes above 256, a bf16 sum would round before the division)
    # (16-bit types only: a float64 gradient stays float64, float32 is already fp32)
    gs = g.float() if g.dtype in (torch.bfloat16, torch.float16) else g
    d = torch.ops.aerognn.scatter_sum(gs, index, ctx.n, False)
    cnt = (rowptr[1:] - rowptr[:-1]).clamp(min=1).to(gs.dtype)
    return (d / cnt[:, None]).to(g.dtype), None, None


torch.library.register_autograd("aerognn::gather_rows", _gather_bwd, setup_context=_gather_ctx)


# ------------------------------------------------------------------------------- scatter_max
@torch.library.custom_op("aerognn::scatter_max", mutates_args=())
def scatter_max(src: Tensor, index: Tensor, dim_size: int) -> tuple[Tensor, Tensor]:
    require_device(src, index)
    src = _rows2d(src, "scatter_max")
    if index.numel() != src.shape[0]:
        raise ValueError("scatter_max: index must have one entry per row of src")
    perm, rowptr = _groups(index, dim_size)
    k = src.shape[1]
    out = torch.empty(dim_size, k, dtype=src.dtype, device=src.device)
    arg = torch.empty(dim_size, k, dtype=I32, device=src.device)
    if dim_size:
        _segment_max(dim_size, k, rowptr, perm, src, out, arg)
    arg64 = arg.to(torch.int64)
    return out, torch.where(arg64 < 0, torch.full_like(arg64, src.shape[0]), arg64)


@scatter_max.register_fake
def _(src, index, dim_size):
    return src.new_empty(dim_size, src.shape[1]), src.new_empty(dim_size, src.shape[1], dtype=torch.int64)


@torch.library.custom_op("aerognn::scatter_max_backward", mutates_args=())
def scatter_max_backward(grad: Tensor, argmax: Tensor, n: int) -> Tensor:
    require_device(grad, argmax)
    grad = _rows2d(grad, "scatter_max_backward")
    arg = torch.where(argmax >= n, torch.full_like(argmax, -1), argmax).to(I32).contiguous()
    dx = torch.zeros(n, grad.shape[1], dtype=grad.dtype, device=grad.device)
    if grad.shape[0]:
        _segment_max_backward(grad.shape[0], grad.shape[1], arg, grad, dx)
    return dx


@scatter_max_backward.register_fake
def _(grad, argmax, n):
    return grad.new_empty(n, grad.shape[1])


def _scatter_max_ctx(ctx, inputs, output):
    src, index, dim_size = inputs
    ctx.save_for_backward(output[1])
    ctx.n = src.shape[0]
    ctx.set_materialize_grads(True)


def _scatter_max_bwd(ctx, g_out, g_arg):
    (arg,) = ctx.saved_tensors
    return torch.ops.aerognn.scatter_max_backward(g_out, arg, ctx.n), None, None


torch.library.register_autograd("aerognn::scatter_max", _scatter_max_bwd, setup_context=_scatter_max_ctx)


# ------------------------------------------------------------------------------- edge_features
@torch.library.custom_op("aerognn::edge_features", mutates_args=())
def edge_features(pos: Tensor, edge_index: Tensor, mean: Optional[Tensor] = None,
                  std: Optional[Tensor] = None) -> Tensor:
    from .data import compute_edge_attr
    if (mean is None) != (std is None):
        raise ValueError("edge_features: give both mean and std, or neither")
    stats = None if mean is None else {"edge_mean": mean, "edge_std": std}
    return compute_edge_attr(pos=pos, edge_index=edge_index, stats=stats)


@edge_features.register_fake
def _(pos, edge_index, mean=None, std=None):
    return pos.new_empty(edge_index.shape[1], pos.shape[1] + 1, dtype=torch.float32)


# ------------------------------------------------------------------------------- PyG-style pools
def global_add_pool(x: Tensor, batch: Optional[Tensor], size: Optional[int] = None) -> Tensor:
    """torch_geometric.nn.global_add_pool on torch.ops.aerognn.scatter_sum."""
    if batch is None:
        batch = torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)
    size = int(batch.max()) + 1 if size is None else size
    return torch.ops.aerognn.scatter_sum(x, batch, size, False)


def global_mean_pool(x: Tensor, batch: Optional[Tensor], size: Optional[int] = None) -> Tensor:
    if batch is None:
        batch = torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)
    size = int(batch.max()) + 1 if size is None else size
    return torch.ops.aerognn.scatter_sum(x, batch, size, True)


def global_max_pool(x: Tensor, batch: Optional[Tensor], size: Optional[int] = None) -> Tensor:
    if batch is None:
        batch = torch.zeros(x.shape[0], dtype=torch.int64, device=x.device)
    size = int(batch.max()) + 1 if size is None else size
    return torch.ops.aerognn.scatter_max(x, batch, size)[0]
