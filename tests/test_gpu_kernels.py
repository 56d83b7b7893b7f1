"""GPU unit tests of individual libaerognn kernels against plain PyTorch references
(float32 / int64 on the device): weight-gradient GEMMs, column sums, radix sort, grouped
segment sums and row gathers, at ragged sizes and with empty segments."""
import os

import pytest
import torch

from golden_util import rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,M,K", [(1, 4, 128), (63, 128, 6), (1000, 128, 128), (70001, 128, 128),
                                      (5000, 256, 128), (12345, 32, 32)])
def test_wgrad_vs_torch(dtype, rows, M, K):
    from aerognn.core import WGrad
    g = torch.Generator(device="cpu").manual_seed(rows)
    G = torch.randn(rows, M, generator=g).to(DEV, dtype)
    X = torch.randn(rows, K, generator=g).to(DEV, dtype)
    dw = torch.empty(M, K, dtype=torch.float32, device=DEV)
    db = torch.empty(M, dtype=torch.float32, device=DEV)
    wg = WGrad()
    wg.add(G, X, dw, db)
    wg.run()
    ref = G.double().t() @ X.double()
    assert rel_l2(dw, ref) <= 1e-6
    assert rel_l2(db, G.double().sum(0)) <= 1e-6


def test_wgrad_split_columns():
    """dW of a concatenated input written into column slices (NodeBlock layer 0: [x, agg])."""
    from aerognn.core import WGrad
    G = torch.randn(3000, 128, device=DEV)
    X1 = torch.randn(3000, 128, device=DEV)
    X2 = torch.randn(3000, 128, device=DEV)
    dw = torch.empty(128, 256, device=DEV)
    wg = WGrad()
    wg.add(G, X1, dw[:, :128])
    wg.add(G, X2, dw[:, 128:])
    wg.run()
    ref = G.double().t() @ torch.cat([X1, X2], 1).double()
    assert rel_l2(dw, ref) <= 1e-6


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("rows,N,K", [(1, 5, 128), (70001, 3000, 128), (999, 50, 6)])
def test_wgrad_gathered_operand(dtype, rows, N, K):
    """agn_wgrad's xidx: X row r = x[idx[r]] (the concat edge MLP's x_src / x_dst blocks) equals
    the product with the materialised x[idx] (ragged stage, repeated indices, narrow K)."""
    from aerognn.core import WGrad
    g = torch.Generator(device="cpu").manual_seed(rows + K)
    G = torch.randn(rows, 128, generator=g).to(DEV, dtype)
    x = torch.randn(N, K, generator=g).to(DEV, dtype)
    idx = torch.randint(0, N, (rows,), generator=g, dtype=torch.int32).to(DEV)
    dw = torch.empty(128, K, dtype=torch.float32, device=DEV)
    db = torch.empty(128, dtype=torch.float32, device=DEV)
    dw2 = torch.empty_like(dw)
    wg = WGrad()
    wg.add(G, x, dw, db, xidx=idx)
    wg.add(G, x.index_select(0, idx.long()).contiguous(), dw2)
    wg.run()
    assert torch.equal(dw, dw2)  # same operand values, same order: bitwise
    ref = G.double().t() @ x.double()[idx.long()]
    assert rel_l2(dw, ref) <= 1e-6 and rel_l2(db, G.double().sum(0)) <= 1e-6


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("with_base", [True, False])
def test_segment_sum2_vs_torch(dtype, with_base):
    """agn_segment_sum2: out = base + sum over src groups (via perm) + sum over dst groups, in
    place over base, against index_add_ in fp64 (empty groups, isolated nodes)."""
    from aerognn.core import segment_sum2
    from aerognn.graph import Level
    g = torch.Generator(device="cpu").manual_seed(7)
    N, E, H = 2000, 9000, 128
    ei = torch.randint(0, N - 100, (2, E), generator=g)  # nodes >= N-100 have no edges
    lv = Level.from_edge_index(ei.to(DEV), N)
    ds = torch.randn(E, H, generator=g)
    dd = torch.randn(E, H, generator=g)
    base = torch.randn(N, H, generator=g)
    # ds / dd rows are the level's (CSC-ordered) edges: row j belongs to src[j] and dst[j]
    src, dst = lv.src.long().cpu(), lv.dst.long().cpu()
    ref = (base.double() if with_base else torch.zeros(N, H, dtype=torch.float64))
    ref = ref.index_add(0, src, ds.double()).index_add(0, dst, dd.double())
    if dtype == torch.float32:  # bitwise the composition it replaces: two segment sums, then (base + A) + B
        from aerognn.core import segment_sum
        A = segment_sum(N, H, lv.rowptr_src, lv.perm_src, ds.to(DEV), torch.empty(N, H, device=DEV))
        B = segment_sum(N, H, lv.rowptr, None, dd.to(DEV), torch.empty(N, H, device=DEV))
        comp = (base.to(DEV) + A) + B if with_base else A + B
    b = base.to(DEV, dtype)
    out = b if with_base else torch.empty(N, H, dtype=dtype, device=DEV)
    segment_sum2(N, H, b if with_base else None, (lv.rowptr_src, lv.perm_src, ds.to(DEV, dtype)),
                 (lv.rowptr, None, dd.to(DEV, dtype)), out)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert rel_l2(out.cpu(), ref) <= tol
    if dtype == torch.float32:
        assert torch.equal(out, comp)


@pytest.mark.parametrize("nw,n", [(1, 256), (47000, 256), (5, 7)])
def test_colsum(nw, n):
    from aerognn.core import colsum_rows
    p = torch.randn(nw, n, device=DEV)
    out = torch.empty(n, device=DEV)
    colsum_rows(p, nw, n, out)
    assert rel_l2(out, p.double().sum(0)) <= 1e-6


@pytest.mark.parametrize("n,bits", [(1, 8), (2047, 20), (2049, 33), (300000, 40), (1000000, 24)])
def test_radix_sort_stable(n, bits):
    from aerognn.graph import radix_sort
    g = torch.Generator(device="cpu").manual_seed(n)
    keys = torch.randint(0, 1 << min(bits, 62), (n,), generator=g, dtype=torch.int64)
    keys = keys // 7 * 7  # many duplicates -> stability matters
    k = keys.to(DEV)
    v = torch.arange(n, dtype=torch.int32, device=DEV)
    radix_sort(k, v, bits)
    ks, order = torch.sort(keys, stable=True)
    assert torch.equal(k.cpu(), ks)
    assert torch.equal(v.cpu().long(), order)


def test_group_by_and_level():
    from aerognn.graph import Level
    g = torch.Generator(device="cpu").manual_seed(0)
    N, E = 500, 4000
    ei = torch.randint(0, N, (2, E), generator=g)
    ei[1, :50] = 7  # one high-degree receiver; some nodes have no edges
    lv = Level.from_edge_index(ei.to(DEV), N)
    perm = lv.perm.cpu()
    assert torch.equal(ei[1][perm], torch.sort(ei[1], stable=True).values)
    assert torch.equal(perm, torch.sort(ei[1], stable=True).indices)
    rp = lv.rowptr.cpu().long()
    assert torch.equal(rp[1:] - rp[:-1], torch.bincount(ei[1], minlength=N))
    ps = lv.perm_src.cpu().long()
    assert torch.equal(lv.src.cpu().long()[ps], torch.sort(lv.src.cpu().long(), stable=True).values)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_segment_sum_and_gather(dtype):
    from aerognn.core import gather_rows, segment_sum
    g = torch.Generator(device="cpu").manual_seed(1)
    rows, n_src, k = 300, 2000, 128
    counts = torch.randint(0, 12, (rows,), generator=g)
    counts[::17] = 0
    ptr = torch.zeros(rows + 1, dtype=torch.int32)
    ptr[1:] = torch.cumsum(counts, 0)
    tot = int(ptr[-1])
    perm = torch.randint(0, n_src, (tot,), generator=g, dtype=torch.int32)
    src = torch.randn(n_src, k, generator=g).to(dtype)
    out = torch.empty(rows, k, dtype=dtype, device=DEV)
    segment_sum(rows, k, ptr.to(DEV), perm.to(DEV), src.to(DEV), out)
    ref = torch.zeros(rows, k, dtype=torch.float64)
    for r in range(rows):
        ref[r] = src[perm[ptr[r]:ptr[r + 1]].long()].double().sum(0)
    tol = 1e-6 if dtype == torch.float32 else 1e-2
    assert rel_l2(out.cpu(), ref) <= tol
    outm = torch.empty_like(out)
    segment_sum(rows, k, ptr.to(DEV), perm.to(DEV), src.to(DEV), outm, mean=True)
    refm = ref / counts.clamp(min=1).double()[:, None]
    assert rel_l2(outm.cpu(), refm) <= tol
    idx = torch.randint(0, rows, (777,), generator=g, dtype=torch.int32)
    add = torch.randn(777, k, generator=g).to(dtype)
    o2 = torch.empty(777, k, dtype=dtype, device=DEV)
    gather_rows(777, k, idx.to(DEV), out, o2, cnt_ptr=ptr.to(DEV), add=add.to(DEV))
    ref2 = out.cpu().double()[idx.long()] / counts.clamp(min=1).double()[idx.long()][:, None] + add.double()
    assert rel_l2(o2.cpu(), ref2) <= tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("with_perm", [True, False])
def test_segment_sum_and_gather_fast_paths_bitwise(dtype, with_perm):
    """The 4-rows-in-flight kernels for 128-wide 16-bit rows (segment_sum4_kernel,
    gather_rows4_kernel) against the general kernels, which an output row stride that is not a
    multiple of 8 elements selects: bitwise (the same fp32 adds in index order)."""
    from aerognn.core import gather_rows, segment_sum
    g = torch.Generator(device="cpu").manual_seed(7)
    rows, n_src, k = 70001, 300000, 128
    counts = torch.randint(0, 14, (rows,), generator=g)
    counts[::13] = 0
    counts[5] = 300
    ptr = torch.zeros(rows + 1, dtype=torch.int32)
    ptr[1:] = torch.cumsum(counts, 0)
    tot = int(ptr[-1])
    perm = torch.randint(0, n_src, (tot,), generator=g, dtype=torch.int32).to(DEV) if with_perm else None
    src = torch.randn(n_src if with_perm else tot, k, generator=g).to(dtype).to(DEV)
    for mean in (False, True):
        fast = torch.empty(rows, k, dtype=dtype, device=DEV)
        gen = torch.empty(rows, k + 2, dtype=dtype, device=DEV)[:, :k]
        segment_sum(rows, k, ptr.to(DEV), perm, src, fast, mean=mean)
        segment_sum(rows, k, ptr.to(DEV), perm, src, gen, mean=mean)
        torch.cuda.synchronize()
        assert torch.equal(fast, gen)
    idx = torch.randint(0, rows, (100003,), generator=g, dtype=torch.int32).to(DEV)
    add = torch.randn(100003, k, generator=g).to(dtype).to(DEV)
    for cnt, ad in ((None, None), (ptr.to(DEV), add)):
        o_fast = torch.empty(100003, k, dtype=dtype, device=DEV)
        o_gen = torch.empty(100003, k + 2, dtype=dtype, device=DEV)[:, :k]
        gather_rows(100003, k, idx, fast, o_fast, cnt_ptr=cnt, add=ad)
        gather_rows(100003, k, idx, fast, o_gen, cnt_ptr=cnt, add=ad)
        torch.cuda.synchronize()
        assert torch.equal(o_fast, o_gen)


@pytest.mark.parametrize("n", [1, 5, 4096, 4097, 300001, 2_000_000])
def test_exclusive_scan(n):
    from aerognn.graph import exclusive_scan
    g = torch.Generator(device="cpu").manual_seed(n)
    x = torch.randint(0, 50, (n,), generator=g, dtype=torch.int32)
    out = exclusive_scan(x.to(DEV)).cpu().long()
    ref = torch.zeros(n + 1, dtype=torch.long)
    ref[1:] = torch.cumsum(x.long(), 0)
    assert torch.equal(out, ref)
