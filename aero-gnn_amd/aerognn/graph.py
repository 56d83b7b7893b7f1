"""Device-side graph levels: receiver-grouped (CSC) edge layout, sender grouping (CSR), and
the bi-stride pooling hierarchy of models/bsms_mgn.py:217-301.

Edge latents of a level are kept in CSC order (edges grouped by receiver `col`, stable in
the reference's own edge order), so the NodeBlock aggregation (mgnLayer.py:144-146) is a
contiguous segmented sum in exactly torch_scatter's summation order. Only integer work
happens here; all of it runs in libaerognn kernels (radix sort, scans, rank sorts).
"""
from __future__ import annotations

import torch

from . import _lib as L
from ._lib import check, ptr
from .core import stream

I32 = torch.int32
I64 = torch.int64


def _bits(n: int) -> int:
    return max(1, int(n - 1).bit_length()) if n > 1 else 1


def radix_sort(keys_u64: torch.Tensor, vals_i32: torch.Tensor, bits: int):
    """Stable sort of (keys, vals) in place on the low `bits` key bits (int64 tensor as u64)."""
    n = keys_u64.numel()
    if n <= 1:
        return keys_u64, vals_i32
    kt = torch.empty_like(keys_u64)
    vt = torch.empty_like(vals_i32)
    scratch = torch.empty(int(L.lib().agn_radix_sort_temp_bytes(n)), dtype=torch.uint8, device=keys_u64.device)
    check(L.lib().agn_radix_sort_u64(ptr(keys_u64), ptr(vals_i32), n, bits, ptr(kt), ptr(vt), ptr(scratch),
                                     stream()), "radix_sort")
    return keys_u64, vals_i32


def group_by(keys: torch.Tensor, nrows: int):
    """Stable grouping of positions 0..n-1 by key (int32, or an int64 row such as edge_index[1]):
    returns (perm int32, rowptr int32 [nrows+1])."""
    n = keys.numel()
    dev = keys.device
    k = torch.empty(n, dtype=I64, device=dev)
    v = torch.empty(n, dtype=I32, device=dev)
    if n:
        k32, k64 = (keys, None) if keys.dtype == I32 else (None, keys)
        check(L.lib().agn_iota_keys(n, ptr(k32), ptr(k64), ptr(k), ptr(v), stream()), "iota_keys")
    radix_sort(k, v, _bits(nrows))
    rp = torch.empty(nrows + 1, dtype=I32, device=dev)
    check(L.lib().agn_row_ptr_i64(ptr(k), n, nrows, ptr(rp), stream()), "row_ptr_i64")
    return v, rp


def exclusive_scan(x: torch.Tensor):
    out = torch.empty(x.numel() + 1, dtype=I32, device=x.device)
    scr = torch.empty(int(L.lib().agn_scan_temp_bytes(x.numel())) // 4 + 1, dtype=I32, device=x.device)
    check(L.lib().agn_exclusive_scan_i32(ptr(x), ptr(out), x.numel(), ptr(out[x.numel():]), ptr(scr), stream()),
          "scan")
    return out


class Level:
    """One graph level in CSC order.

    src/dst: int32 [E] (CSC order), rowptr: int32 [N+1] grouping by receiver,
    perm_src/rowptr_src: sender grouping (positions into the CSC edge list),
    refkey: int64 [E], the edge's position in the REFERENCE's own edge order at this level
    (caller's order at level 0; (row, col) lexicographic at coarse levels, bsms_mgn.py:280),
    perm: int64 [E] caller edge id of each CSC edge (level 0 only).
    """

    def __init__(self, N, src, dst, rowptr, refkey, perm=None):
        self.N = int(N)
        self.E = int(src.numel())
        self.src, self.dst, self.rowptr = src, dst, rowptr
        self.refkey = refkey
        self.perm = perm
        self.perm_src, self.rowptr_src = group_by(src, self.N)
        self._perm_inv = None

    @property
    def perm_inv(self):
        if self._perm_inv is None and self.perm is not None:
            inv = torch.empty_like(self.perm)
            inv[self.perm] = torch.arange(self.perm.numel(), device=self.perm.device)
            self._perm_inv = inv
        return self._perm_inv

    @staticmethod
    def from_edge_index(edge_index: torch.Tensor, N: int) -> "Level":
        """Reference edge_index [2,E] int64 (any order) -> CSC level (stable by edge id), all in
        libaerognn kernels: radix sort of the receivers, row pointers, one gather pass."""
        ei = edge_index if edge_index.dtype == I64 and edge_index.stride(1) == 1 else edge_index.to(I64).contiguous()
        E = ei.shape[1]
        dev = ei.device
        perm32, rowptr = group_by(ei[1], N)
        src = torch.empty(E, dtype=I32, device=dev)
        dst = torch.empty(E, dtype=I32, device=dev)
        perm = torch.empty(E, dtype=I64, device=dev)
        inv = torch.empty(E, dtype=I64, device=dev)
        inv32 = torch.empty(E, dtype=I32, device=dev)
        check(L.lib().agn_level_index(E, ptr(ei), ei.stride(0), ptr(perm32), ptr(src), ptr(dst), ptr(perm), ptr(inv),
                                      ptr(inv32), stream()), "level_index")
        lv = Level(N, src, dst, rowptr, perm, perm=perm)
        lv._perm_inv = inv
        lv.perm32, lv.inv32 = perm32, inv32  # the row permutations caller <-> CSC (PermuteRowsFn)
        return lv


class Pooling:
    """Index maps of one bi-stride downsampling step (bsms_mgn.py:217-301), fine -> coarse.

    f2c int32 [N] (the reference's `fine_to_coarse`), c2f/c2f_ptr (coarse members in
    ascending fine id), cbatch int64 [Nc], coarse Level (CSC), cand_sorted/cmem_ptr (fine
    edges of each coarse edge in reference order), inv int32 [E] (fine edge -> coarse edge).
    """
    pass


def downsample_maps(level: Level, batch, pos, stride: int, ngraph: int) -> Pooling:
    dev = level.src.device
    n = level.N
    P = Pooling()
    lib = L.lib()
    # 1. order nodes by (graph, x) — per-graph argsort(pos[:, 0]) with the stable tie rule
    if pos is not None:
        pos32 = pos if pos.dtype == torch.float32 else pos.float()
        pos32 = pos32.contiguous()
        keys = torch.empty(n, dtype=I64, device=dev)
        sorted_nodes = torch.empty(n, dtype=I32, device=dev)
        check(lib.agn_pool_sort_keys(n, ptr(batch), ptr(pos32), pos32.stride(0), ptr(keys), ptr(sorted_nodes),
                                     stream()), "pool_sort_keys")
        radix_sort(keys, sorted_nodes, 32 + (_bits(ngraph) if ngraph > 1 else 0))
    else:
        sorted_nodes = torch.arange(n, dtype=I32, device=dev)  # node order (bsms_mgn.py:244-245)
    # 2. graph starts, coarse offsets (torch on G+1 ints: plumbing)
    if batch is not None:
        gstart = torch.empty(ngraph + 1, dtype=I32, device=dev)
        check(lib.agn_row_ptr_i64(ptr(batch), n, ngraph, ptr(gstart), stream()), "row_ptr_i64")
    else:
        gstart = torch.tensor([0, n], dtype=I32, device=dev)
    cnt = (gstart[1:] - gstart[:-1] + (stride - 1)) // stride
    coff = torch.zeros(ngraph + 1, dtype=I32, device=dev)
    coff[1:] = torch.cumsum(cnt, 0)
    nc = int(coff[-1].item())  # host sync (the reference syncs per graph, bsms_mgn.py:234,250)
    P.nc = nc
    P.f2c = torch.empty(n, dtype=I32, device=dev)
    P.c2f = torch.empty(n, dtype=I32, device=dev)
    P.c2f_ptr = torch.empty(nc + 1, dtype=I32, device=dev)
    P.cbatch = torch.empty(nc, dtype=I64, device=dev)
    check(lib.agn_pool_assign(n, nc, ngraph, ptr(batch), ptr(sorted_nodes), ptr(gstart), ptr(coff), stride,
                              ptr(P.f2c), ptr(P.c2f), ptr(P.c2f_ptr), ptr(P.cbatch), stream()), "pool_assign")
    # 3. coarse edges: per coarse receiver, rank-sort member edges by (f2c[src], ref order)
    cand_cnt = torch.empty(nc, dtype=I32, device=dev)
    check(lib.agn_pool_edge_candidates(nc, ptr(P.c2f), ptr(P.c2f_ptr), ptr(level.rowptr), ptr(cand_cnt), stream()),
          "pool_edge_candidates")
    cand_ptr = exclusive_scan(cand_cnt)
    cand_tmp = torch.empty(level.E, dtype=I32, device=dev)
    P.cand_sorted = torch.empty(level.E, dtype=I32, device=dev)
    uniq = torch.empty(nc, dtype=I32, device=dev)
    check(lib.agn_pool_edge_sort(nc, ptr(P.c2f), ptr(P.c2f_ptr), ptr(level.rowptr), ptr(level.src),
                                 ptr(level.refkey), ptr(P.f2c), ptr(cand_ptr), ptr(cand_tmp), ptr(P.cand_sorted),
                                 ptr(uniq), stream()), "pool_edge_sort")
    crowptr = exclusive_scan(uniq)
    ec = int(crowptr[-1].item())  # host sync (reference: torch.unique, bsms_mgn.py:280)
    csrc = torch.empty(ec, dtype=I32, device=dev)
    cdst = torch.empty(ec, dtype=I32, device=dev)
    P.cmem_ptr = torch.empty(ec + 1, dtype=I32, device=dev)
    P.inv = torch.empty(level.E, dtype=I32, device=dev)
    crefkey = torch.empty(ec, dtype=I64, device=dev)
    check(lib.agn_pool_edge_emit(nc, ptr(cand_ptr), ptr(P.cand_sorted), ptr(level.src), ptr(P.f2c), ptr(crowptr),
                                 ptr(csrc), ptr(cdst), ptr(P.cmem_ptr), ptr(P.inv), ptr(crefkey), level.E, stream()),
          "pool_edge_emit")
    P.coarse = Level(nc, csrc, cdst, crowptr, crefkey)
    return P
