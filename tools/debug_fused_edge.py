"""Diagnostics (GPU, not a test): agn_edge_bwd_fused against the split path on one C3-like layer.

Runs the edge chain's forward with saves, then the split backward (agn_mlp_backward) and the
fused backward on the same synthetic upstream gradients, and reports where G0 and de differ.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aerognn import core
    from aerognn import _lib as L
    from aerognn.functions import _alloc_saves, _alloc_gpre
    from aerognn.graph import Level
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    dev = "cuda"
    m = ellipsoid(150, 110, seed=0)
    ei = torch.from_numpy(np.ascontiguousarray(m["edge_index"])).to(dev)
    N, E, H = m["x"].shape[0], ei.shape[1], 128
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).to(dev)
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(N, H, generator=g).to(dev, torch.bfloat16)
    e = torch.randn(E, H, generator=g).to(dev, torch.bfloat16)
    ge = torch.randn(E, H, generator=g).to(dev, torch.bfloat16)
    dagg = torch.randn(N, H, generator=g).to(dev, torch.bfloat16)
    spec = layer.spec()
    spec.pack.update(torch.bfloat16, dev)
    es = spec.edge
    dt = torch.bfloat16
    P = torch.empty(N, 2 * H, dtype=dt, device=dev)
    core.proj_forward(N, x, spec.pack["proj"], spec.pack["proj_b"], P)
    ea, ehp, est = _alloc_saves(es, E, dt, dev, True)
    e_out = torch.empty_like(e)
    core.mlp_forward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, out_dim=H,
                     segs=[(L.SEG_PLAIN, H, e.stride(0), e, None, None)], wpk=es.wpk(), bias=es.biases(),
                     ln=es.lnp(), proj=P, src=lv.src, dst=lv.dst, resid=e, out=e_out, acts=ea, hpre=ehp, stats=est)
    gpre = _alloc_gpre(es, E, dt, dev, rowmajor=(0, 1, 2, 3))
    de_s = torch.empty_like(e)
    nb = core.bwd_nblocks(E)
    part = torch.empty(nb, 2 * H, dtype=torch.float32, device=dev)
    core.mlp_backward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, out_dim=H, in_dim=H, wtpk=es.wtpk(), acts=ea, g=ge,
                      g2=dagg, gidx=lv.dst, gpre=gpre, ln_g=es.lnp()[0], hpre=ehp, stats=est, din=[(H, de_s, True)],
                      ln_partial=part)
    de_f = torch.empty_like(e)
    g0_f = torch.empty(E, H, dtype=dt, device=dev)
    dW, db, lnp, nblk = core.edge_bwd_fused(rows=E, wpk=es.wpk(), wtpk0=es.wtpk()[0], bias=es.biases(), ln_g=es.lnp()[0], e=e, proj=P,
                                            src=lv.src, dst=lv.dst, g=ge, g2=dagg, de=de_f, g0=g0_f)
    torch.cuda.synchronize()
    for name, a, b in (("G0", g0_f, gpre[0]), ("de", de_f, de_s)):
        d = (a != b)
        rows = d.any(1).nonzero().flatten()
        feats = d.any(0).nonzero().flatten()
        print(f"{name}: differing {int(d.sum())} of {d.numel()}; rows {rows.numel()} (first {rows[:8].tolist()}), "
              f"features {feats.numel()} (first {feats[:16].tolist()})")
        if rows.numel():
            r = int(rows[0])
            f = d[r].nonzero().flatten()[:6]
            print("   row", r, "fused", a[r, f].float().tolist(), "split", b[r, f].float().tolist())
            tiles = torch.unique(rows // 32)
            print("   tiles", tiles.numel(), "rows-in-tile", torch.unique(rows % 32)[:32].tolist())
    # dW vs the split path's wgrad
    wg = core.WGrad()
    dws = [torch.empty(H, H, dtype=torch.float32, device=dev) for _ in range(3)]
    dbs = [torch.empty(H, dtype=torch.float32, device=dev) for _ in range(3)]
    for l in range(3):
        wg.add(gpre[l + 1], ea[l], dws[l], dbs[l])
    wg.run()
    torch.cuda.synchronize()
    for l in range(3):
        r = float((dW[l] - dws[l]).norm() / dws[l].norm())
        rb = float((db[l] - dbs[l]).norm() / dbs[l].norm())
        print(f"dW{l + 1} rel-L2 {r:.3e}   db{l + 1} rel-L2 {rb:.3e}")


if __name__ == "__main__":
    main()
