"""float64 references for the bf16 MLP-chain kernels, run through the kernels' OWN saves (test
infrastructure, not product code; DESIGN.md §4 "mask-matched").

A bf16 chain kernel rounds every activation and every pre-activation gradient to bf16. Against an
independent float64 model those roundings flip ReLU kinks (~0.2 % of the inputs), and each flip moves
its gradient element by O(1), which forces loose (~1e-1) gates. Here the float64 side instead takes
the kernel's saved bf16 activations as the inputs of each layer (forward: each layer's float64
product from the kernel's previous activation, rounded once, must equal the kernel's activation up
to fp32-accumulation ties at bf16 rounding boundaries) and its ReLU masks in the backward, so what
remains is the kernel's bf16 rounding of each G_l (~1e-3 per rounding): the gates can sit at 3x the
measured values, near bf16 rounding.

Reference chain: models/mlp.py:40-51 (Linear -> act -> ... -> Linear -> LayerNorm), the NodeBlock /
EdgeBlockSum residuals of models/mgnLayer.py:153,205.
"""
import torch

H = 128


def bf(t):
    """fp64 of the bf16 rounding of t."""
    return t.to(torch.bfloat16).to(torch.float64)


def decode_tiled(t, rows, width=H):
    """AGN_TILED [rows_pad, 128] 16-bit -> row-major [rows, 128] (aerognn.h: unit (i, h) of row c
    holds features 16i+4h+{0..3}, 16i+8+4h+{0..3})."""
    assert width == H
    u = t.view(torch.int16).reshape(-1, 8, 2, 32, 8)  # [tile][i][h][c][8]
    out = torch.empty(u.shape[0], 32, H, dtype=torch.int16, device=t.device)
    for i in range(8):
        for hh in range(2):
            v = u[:, i, hh]
            out[:, :, 16 * i + 4 * hh:16 * i + 4 * hh + 4] = v[:, :, :4]
            out[:, :, 16 * i + 8 + 4 * hh:16 * i + 8 + 4 * hh + 4] = v[:, :, 4:]
    return out.reshape(-1, H)[:rows].view(t.dtype)


def rows_of(t, rows):
    """A save as row-major [rows, w] (decoding AGN_TILED buffers)."""
    if getattr(t, "agn_tiled", False):
        return decode_tiled(t, rows)
    return t[:rows]


def check_bf16_layer(name, got, ref64, relu, max_frac=1e-4):
    """got (bf16) vs round(ref64) (with relu): equal except where the fp32 accumulation (absolute
    error ~1e-6 on O(1) sums) lands on the other side of a bf16 rounding boundary: a few elements per
    million, each within one ulp of the rounded value or within 1e-4 absolute (tiny values)."""
    want = ref64.clamp_min(0.0) if relu else ref64
    want = want.to(torch.bfloat16)
    diff = got.view(torch.int16) != want.view(torch.int16)
    frac = diff.double().mean().item()
    worst = 0.0
    if frac:
        g, w = got[diff].double(), want[diff].double()
        ulp = (w.abs() * 2.0 ** -7).clamp_min(2.0 ** -133)
        worst = ((g - w).abs() / torch.maximum(ulp, torch.full_like(ulp, 1e-4))).max().item()
    print(f"  forward {name}: {frac:.2e} of the elements differ from the rounded float64 value "
          f"(worst {worst:.2f} of max(1 ulp, 1e-4))")
    assert frac <= max_frac and worst <= 1.0, (name, frac, worst)


def chain_forward_check(X, W, b, acts, hpre, stats, ln, out=None, resid=None, tag=""):
    """Layer-by-layer forward check of a chain from its saves. X: the chain input (fp64 of the
    kernel's bf16 operand rows); W: fp64 bf16-rounded weights; b: fp64 biases (fp32 values);
    acts: the kernel's bf16 ReLU outputs (row-major); hpre / stats: its pre-LN rows and (mean, rstd)
    (LayerNorm chains) or None; out: the kernel output, checked against round(round(LN(h)) + resid)
    (or round(h) without LayerNorm)."""
    prev = X
    nlin = len(W)
    for l in range(nlin - 1):
        h = prev @ W[l].T + b[l]
        check_bf16_layer(f"{tag}a{l + 1}", acts[l], h, True)
        prev = acts[l].double()
    h = prev @ W[-1].T + b[-1]
    from golden_util import rel_l2
    if ln is None:
        if out is not None:
            check_bf16_layer(f"{tag}out", out, h, False)
        return
    check_bf16_layer(f"{tag}h{nlin - 1} (pre-LN)", hpre, h, False)
    mean = h.mean(1)
    rstd = 1.0 / torch.sqrt(((h - mean[:, None]) ** 2).mean(1) + 1e-5)
    rm = rel_l2(stats[:, 0].double(), mean)
    rr = rel_l2(stats[:, 1].double(), rstd)
    print(f"  forward {tag}LayerNorm statistics: mean rel-L2 {rm:.2e}, rstd {rr:.2e}")
    assert rm <= 1e-5 and rr <= 1e-5
    if out is not None:
        y = bf((h - mean[:, None]) * rstd[:, None] * ln[0] + ln[1])
        ref = bf(y + resid) if resid is not None else y
        r = rel_l2(out.double(), ref)
        print(f"  forward {tag}out: rel-L2 {r:.2e} against round(round(LN(h)) + residual)")
        assert r <= 5e-3


def chain_backward_ref(X, W, acts, g, ln=None, hpre=None, stats=None):
    """float64 backward through the kernel's masks and saves. g: gradient of the chain output
    (before any residual); returns G_0..G_{n-1}, dX (= G_0 W_0), dW_l, db_l, (dgamma, dbeta)."""
    A = [a.double() for a in acts]
    nlin = len(W)
    out = {}
    if ln is not None:
        mean, rstd = stats[:, 0].double(), stats[:, 1].double()
        xh = (hpre.double() - mean[:, None]) * rstd[:, None]
        gg = g * ln[0]
        c1 = gg.mean(1, keepdim=True)
        c2 = (gg * xh).mean(1, keepdim=True)
        G = (gg - c1 - xh * c2) * rstd[:, None]
        out["dgamma"], out["dbeta"] = (g * xh).sum(0), g.sum(0)
    else:
        G = g
    Gs = [None] * nlin
    Gs[-1] = G
    for l in range(nlin - 1, 0, -1):
        Gs[l - 1] = (Gs[l] @ W[l]) * (A[l - 1] > 0)
    ins = [X] + A
    for l in range(nlin):
        out[f"G{l}"] = Gs[l]
        out[f"dW{l}"] = Gs[l].T @ ins[l]
        out[f"db{l}"] = Gs[l].sum(0)
    out["dX"] = Gs[0] @ W[0]
    return out


def gate(results, measured, label):
    """Assert rel-L2 <= 3x measured for every key of `results` ({key: rel-L2})."""
    fails = []
    for k, r in results.items():
        g = 3.0 * measured[k]
        print(f"  {label} {k}: rel-L2 {r:.3e} against the mask-matched float64 backward (gate {g:.1e})")
        if not r <= g:
            fails.append((k, r, g))
    assert not fails, fails
