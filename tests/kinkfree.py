"""Inputs conditioned away from ReLU kinks, for gradient parity at large sizes.

A ReLU's derivative jumps at 0. Where a pre-activation lies within the fp32 rounding band of 0,
the HIP kernels and the CPU oracle (same math, different summation order; forwards agree to
~3e-7) can take different sides, and that one element changes its row's gradient by O(1): at
C2 size (~2e8 edge pre-activations) a handful of such rows put the whole-tensor gradient error
at 1e-4..1e-3 whatever the kernels do (measured: tools/debug_layer_sizes.py). Here every row
whose float64 oracle pre-activation lies within `band` (relative to that layer's spread) of a
kink is re-drawn, until no row does; the gradient comparison at the 1e-5 bar then measures the
kernels, not the coin flips. Rows are re-drawn, never dropped from the comparison.
"""
import torch


def kink_free(layer_fn, x, e, gen, band=1e-5, rounds=8):
    """layer_fn(x64, e64) runs the oracle forward (float64); x, e are re-drawn in place (rows of
    nodes / edges whose MLP pre-activations come within band * std of 0). Returns the number of
    rows re-drawn in total."""
    from oracle import refcpu as R
    redrawn = 0
    for _ in range(rounds):
        near_e, near_x = set(), set()

        def tap(pre, i, h):
            t = h.detach()
            rows = (t.abs() < band * t.std()).any(1).nonzero().flatten().tolist()
            (near_x if "node_block" in pre else near_e).update(rows)
        R.PRE_ACT_TAP = tap
        try:
            with torch.no_grad():
                layer_fn(x.double(), e.double())
        finally:
            R.PRE_ACT_TAP = None
        if not near_e and not near_x:
            return redrawn
        if near_e:
            i = torch.tensor(sorted(near_e))
            e[i] = torch.randn(len(i), e.shape[1], generator=gen, dtype=e.dtype)
        if near_x:
            i = torch.tensor(sorted(near_x))
            x[i] = torch.randn(len(i), x.shape[1], generator=gen, dtype=x.dtype)
        redrawn += len(near_e) + len(near_x)
    raise AssertionError(f"inputs not kink-free after {rounds} rounds")


def _bias_key(p, pre, i):
    """The bias parameter added into pre-activation `i` of the MLP at prefix `pre` (oracle/refcpu.py
    naming: mlp() layers, or EdgeBlockSum's fused first bias / hidden `mlp.{k}` layers)."""
    for k in (f"{pre}.layers.{i}.bias", f"{pre}.mlp.{i}.bias", f"{pre}.bias" if i == 0 else None):
        if k is not None and k in p:
            return k
    raise KeyError(f"no bias for pre-activation {i} of {pre}")


def kink_free_biases(run64, p64, band=2e-5, margin=3.0, rounds=4):
    """Whole-model conditioning: `run64()` runs the float64 oracle forward with the parameter dict
    `p64`. Every ReLU input column holding an element within `band` * (that pre-activation's std) of
    0 gets its bias shifted by the smallest step (multiples of `margin` * band * std) that clears the
    whole column; the shift is applied to the running forward too (h[:, j] += d, which IS the forward
    with the shifted bias), so one pass conditions every layer in execution order. Biases are
    changed, inputs never; a final pass must find no element within band. Returns the number of
    columns shifted."""
    from oracle import refcpu as R
    shifted = 0
    for _ in range(rounds):
        hits = [0]

        def tap(pre, i, h):
            thr = band * float(h.std())
            near = (h.abs() < thr).any(0).nonzero().flatten().tolist()
            if not near:
                return
            key = _bias_key(p64, pre, i)
            steps = torch.tensor([s * margin * thr for k in range(1, 40) for s in (k, -k)], dtype=h.dtype)
            for j in near:
                v = h[:, j]
                ok = ((v[None, :] + steps[:, None]).abs() >= 2 * thr).all(1).nonzero().flatten()
                if len(ok) == 0:
                    raise AssertionError(f"kink_free_biases: no shift clears column {j} of {pre}[{i}]")
                d = steps[int(ok[0])]
                h[:, j] += d
                with torch.no_grad():
                    p64[key][j] += d
            hits[0] += len(near)
        R.PRE_ACT_TAP = tap
        try:
            with torch.no_grad():
                run64()
        finally:
            R.PRE_ACT_TAP = None
        if hits[0] == 0:
            return shifted
        shifted += hits[0]
    raise AssertionError(f"biases not kink-free after {rounds} rounds")
