"""torch.ops.aerognn.* on the MI355X vs torch's CPU ops (aerognn/ops.py).

scatter_sum follows torch_scatter's CPU order (rows added in increasing index), so fp32 sums are
bitwise torch's CPU index_add_; means are sum / count (1 ulp); bf16 accumulates in fp32 and is
compared with the fp32 reference rounded to bf16. scatter_max matches scatter_reduce('amax') with
torch_scatter's argmax convention (first maximal row, n for empty groups). torch.library.opcheck
checks each op's schema, fake kernel and autograd registration."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _data(n=5000, k=24, G=300, seed=0, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, k, generator=g).to(dtype)
    idx = torch.randint(0, G, (n,), generator=g)
    idx[idx == 7] = 8  # an empty group
    return x, idx, G


def test_scatter_sum_matches_torch_cpu():
    import aerognn.ops  # noqa: F401
    x, idx, G = _data()
    ref = torch.zeros(G, x.shape[1]).index_add_(0, idx, x)
    got = torch.ops.aerognn.scatter_sum(x.to(DEV), idx.to(DEV), G, False).cpu()
    assert torch.equal(got, ref)
    cnt = torch.bincount(idx, minlength=G).clamp(min=1).float()
    mean = torch.ops.aerognn.scatter_sum(x.to(DEV), idx.to(DEV), G, True).cpu()
    assert torch.allclose(mean, ref / cnt[:, None], rtol=2e-7, atol=0)
    xb = x.bfloat16()
    refb = torch.zeros(G, x.shape[1]).index_add_(0, idx, xb.float()).bfloat16()
    gotb = torch.ops.aerognn.scatter_sum(xb.to(DEV), idx.to(DEV), G, False).cpu()
    assert (gotb.float() - refb.float()).abs().max() <= 1e-2 * refb.float().abs().max()


def test_gather_rows_and_backward():
    import aerognn.ops  # noqa: F401
    x, idx, G = _data()
    src = torch.randn(G, x.shape[1])
    got = torch.ops.aerognn.gather_rows(src.to(DEV), idx.to(DEV)).cpu()
    assert torch.equal(got, src.index_select(0, idx))
    s = src.to(DEV).requires_grad_(True)
    w = torch.randn(idx.numel(), x.shape[1])
    (torch.ops.aerognn.gather_rows(s, idx.to(DEV)) * w.to(DEV)).sum().backward()
    assert torch.equal(s.grad.cpu(), torch.zeros_like(src).index_add_(0, idx, w))


def test_gather_rows_mean_backward_float64_stays_float64():
    """the mean-gather backward sums and divides a float64 gradient in float64 (only 16-bit
    types are upcast to fp32)."""
    import aerognn.ops  # noqa: F401
    n, k = 5000, 8
    g = torch.Generator().manual_seed(5)
    idx = torch.sort(torch.randint(0, 40, (n,), generator=g)).values
    rowptr = torch.searchsorted(idx, torch.arange(41))
    src = torch.randn(40, k, dtype=torch.float64, generator=g)
    w = torch.randn(n, k, dtype=torch.float64, generator=g)
    s = src.to(DEV).requires_grad_(True)
    (torch.ops.aerognn.gather_rows(s, idx.to(DEV), rowptr.to(DEV)) * w.to(DEV)).sum().backward()
    cnt = (rowptr[1:] - rowptr[:-1]).clamp(min=1).double()
    ref = torch.zeros(40, k, dtype=torch.float64).index_add_(0, idx, w) / cnt[:, None]
    assert s.grad.dtype == torch.float64
    assert torch.allclose(s.grad.cpu(), ref, rtol=1e-13, atol=1e-13)


def test_gather_rows_mean_backward_bf16_large_groups():
    """gather_rows with a group-size divisor (the broadcast side of a mean pool): its backward sums
    and divides in fp32 and rounds once, so a 100,000-row group's gradient is the fp32 value rounded
    to bf16 (a bf16 count would read 99,840)."""
    import aerognn.ops  # noqa: F401
    n, k = 100_000, 8
    idx = torch.zeros(n, dtype=torch.long)
    idx[60_000:] = 1
    rowptr = torch.tensor([0, 60_000, n])
    w = torch.randn(n, k, generator=torch.Generator().manual_seed(3)).bfloat16()
    s = torch.zeros(2, k, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    (torch.ops.aerognn.gather_rows(s, idx.to(DEV), rowptr.to(DEV)).float() * w.to(DEV).float()).sum().backward()
    ref = torch.zeros(2, k).index_add_(0, idx, w.float()) / torch.tensor([60_000.0, 40_000.0])[:, None]
    got = s.grad.cpu().float()
    print("max rel err", float(((got - ref).abs() / ref.abs()).max()))
    assert torch.equal(s.grad.cpu(), ref.bfloat16()) or float(((got - ref).abs() / ref.abs()).max()) <= 2 ** -8


@pytest.mark.parametrize("mean", [False, True])
def test_scatter_sum_backward(mean):
    import aerognn.ops  # noqa: F401
    x, idx, G = _data(n=3000, k=16)
    w = torch.randn(G, x.shape[1])
    xr = x.clone().requires_grad_(True)
    cnt = torch.bincount(idx, minlength=G).clamp(min=1).float()[:, None]
    ref = torch.zeros(G, x.shape[1]).index_add(0, idx, xr)
    ((ref / cnt if mean else ref) * w).sum().backward()
    xg = x.to(DEV).requires_grad_(True)
    (torch.ops.aerognn.scatter_sum(xg, idx.to(DEV), G, mean) * w.to(DEV)).sum().backward()
    assert torch.allclose(xg.grad.cpu(), xr.grad, rtol=1e-6, atol=0)


def test_scatter_max_values_argmax_and_backward():
    import aerognn.ops  # noqa: F401
    x, idx, G = _data(n=4000, k=8)
    x[::13] = x[::13].round()  # ties: the first maximal row wins
    out, arg = torch.ops.aerognn.scatter_max(x.to(DEV), idx.to(DEV), G)
    out, arg = out.cpu(), arg.cpu()
    ref = torch.zeros(G, x.shape[1]).scatter_reduce_(0, idx[:, None].expand_as(x), x, "amax", include_self=False)
    assert torch.equal(out, ref)
    xn, inn = x.numpy(), idx.numpy()
    for r in (0, 7, 8, G - 1):
        rows = np.nonzero(inn == r)[0]
        for f in range(x.shape[1]):
            want = rows[np.argmax(xn[rows, f])] if rows.size else x.shape[0]
            assert int(arg[r, f]) == want, (r, f)
    xg = x.to(DEV).requires_grad_(True)
    w = torch.randn(G, x.shape[1])
    (torch.ops.aerognn.scatter_max(xg, idx.to(DEV), G)[0] * w.to(DEV)).sum().backward()
    dref = torch.zeros_like(x)
    for r in range(G):
        for f in range(x.shape[1]):
            if int(arg[r, f]) < x.shape[0]:
                dref[int(arg[r, f]), f] = w[r, f]
    assert torch.equal(xg.grad.cpu(), dref)


def test_global_pools_match_oracle():
    import aerognn.ops as O
    from oracle import refcpu as R
    x, _, _ = _data(n=2000, k=12)
    batch = torch.repeat_interleave(torch.arange(5), torch.tensor([300, 500, 200, 600, 400]))
    for name, fn in (("add", O.global_add_pool), ("mean", O.global_mean_pool), ("max", O.global_max_pool)):
        got = fn(x.to(DEV), batch.to(DEV)).cpu()
        ref = R.global_pool(x, batch, name)
        assert torch.allclose(got, ref, rtol=2e-7 if name == "mean" else 0, atol=0), name


def test_edge_features_op_matches_data_module():
    import aerognn.ops  # noqa: F401
    from aerognn import data as D
    from aerognn.meshgen import ellipsoid
    m = ellipsoid(30, 20, seed=1)
    pos, ei = torch.from_numpy(m["pos"]).to(DEV), torch.from_numpy(m["edge_index"]).to(DEV)
    assert torch.equal(torch.ops.aerognn.edge_features(pos, ei), D.compute_edge_attr(pos=pos, edge_index=ei))


@pytest.mark.parametrize("name", ["scatter_sum", "gather_rows", "scatter_max"])
def test_opcheck(name):
    import aerognn.ops  # noqa: F401
    x, idx, G = _data(n=600, k=8)
    x, idx = x.to(DEV).requires_grad_(True), idx.to(DEV)
    args = {"scatter_sum": (x, idx, G, True), "gather_rows": (torch.randn(G, 8, device=DEV, requires_grad=True), idx),
            "scatter_max": (x, idx, G)}[name]
    torch.library.opcheck(getattr(torch.ops.aerognn, name).default, args)
