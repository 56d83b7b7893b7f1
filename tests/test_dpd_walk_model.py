"""Host model of the fused backward's dP_d ownership (csrc/edge_bwd.hip dpd_pair / dpd_row /
dpd_cross_kernel), checked against agn_segment_sum's arithmetic (fp32 sum in edge order from
zero) bit for bit over random receiver layouts. No GPU: this pins the protocol, the GPU test
(tests/test_gpu_edge16.py::test_fused_backward_dpd_bitwise_segment_sum) pins the kernel.

The kernel's rules, restated:
* rows are walked in 128-row rounds (4 chain-wave tiles of 32); a round's first row opens a run;
* every row adds its value to the open run (restarted at a change of receiver) and stores the
  running sum to dP_d[dst[row]]; a receiver's last store within the round is its in-round sum;
* afterwards dpd_cross_kernel overwrites every receiver whose rows span a round boundary, and
  every empty receiver, with the full sum (zeros for empty ones).
"""
import numpy as np
import pytest

ROUND = 128


def _segment_sums(dst, vals, n):
    out = np.zeros((n, vals.shape[1]), np.float32)
    for r in range(len(dst)):  # edge order, fp32, from zero (segment_sum_kernel)
        out[dst[r]] = np.float32(out[dst[r]] + vals[r])
    return out


def _kernel_model(dst, vals, n):
    out = np.full((n, vals.shape[1]), np.nan, np.float32)  # never-written marker
    E = len(dst)
    for r0 in range(0, E, ROUND):
        cur, s = -1, None
        for r in range(r0, min(r0 + ROUND, E)):
            s = vals[r].copy() if dst[r] != cur else np.float32(s + vals[r])
            cur = dst[r]
            out[cur] = s
    rowptr = np.zeros(n + 1, np.int64)
    np.add.at(rowptr, dst + 1, 1)
    rowptr = np.cumsum(rowptr)
    for v in range(n):
        beg, end = rowptr[v], rowptr[v + 1]
        if end > beg and beg // ROUND == (end - 1) // ROUND:
            continue  # the fused kernel's
        acc = np.zeros(vals.shape[1], np.float32)
        for j in range(beg, end):
            acc = np.float32(acc + vals[j])
        out[v] = acc
    return out


@pytest.mark.parametrize("seed", range(40))
def test_dpd_walk_model_matches_segment_sum(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 400))
    E = int(rng.integers(1, 1500))
    kind = seed % 4
    if kind == 0:    # uniform receivers
        dst = np.sort(rng.integers(0, n, E))
    elif kind == 1:  # long runs (coarse levels: tens of edges per receiver)
        dst = np.sort(rng.integers(0, max(1, n // 40), E))
    elif kind == 2:  # runs ending on round boundaries
        deg = rng.choice([1, 127, 128, 129, 256], size=max(1, E // 128))
        dst = np.repeat(np.arange(len(deg)) % n, deg)[:E]
        dst = np.sort(dst)
        E = len(dst)
    else:            # sparse: many empty receivers
        dst = np.sort(rng.choice(n, size=E, replace=True) // 3 * 3 % n)
    vals = (rng.standard_normal((E, 4)) * 10.0 ** rng.integers(-3, 3, (E, 1))).astype(np.float32)
    want = _segment_sums(dst, vals, n)
    got = _kernel_model(dst, vals, n)
    assert np.array_equal(got.view(np.int32), want.view(np.int32))
