"""dP_d on the fused backward's dW waves, timed (diagnostic, not the product
path): one C3 level-0 sized layer (1M nodes / ~6M edges, ellipsoid mesh in CSC order), the 32-row
agn_edge_bwd_fused with and without dP_d, and the agn_segment_sum launch dP_d replaces. HIP events
on the launch stream, median of --reps.

Usage (GPU): python tools/dpd_timing.py [--nu 1000] [--reps 7]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nu", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    import numpy as np
    import torch
    from aerognn import core
    from aerognn.graph import Level
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    dev = "cuda"
    m = ellipsoid(args.nu, args.nu, seed=0)
    ei = torch.from_numpy(np.ascontiguousarray(m["edge_index"])).to(dev)
    N, E, H = m["x"].shape[0], ei.shape[1], 128
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).to(dev)
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    dt = torch.bfloat16
    x = torch.randn(N, H, generator=g).to(dev, dt)
    e = torch.randn(E, H, generator=g).to(dev, dt)
    ge = torch.randn(E, H, generator=g).to(dev, dt)
    dagg = torch.randn(N, H, generator=g).to(dev, dt)
    spec = layer.spec()
    spec.pack.update(dt, dev)
    es = spec.edge
    P = torch.empty(N, 2 * H, dtype=dt, device=dev)
    core.proj_forward(N, x, spec.pack["proj"], spec.pack["proj_b"], P)
    de = torch.empty_like(e)
    g0 = torch.empty(E, H, dtype=dt, device=dev)
    dpd = torch.empty(N, H, dtype=dt, device=dev)
    ref = torch.empty(N, H, dtype=dt, device=dev)

    def bwd(with_dpd):
        return lambda: core.edge_bwd_fused(rows=E, wpk=es.wpk(), bias=es.biases(), ln_g=es.lnp()[0], e=e, proj=P,
                                           src=lv.src, dst=lv.dst, g=ge, g2=dagg, de=de, g0=g0,
                                           dpd=dpd if with_dpd else None, rowptr=lv.rowptr)

    def seg():
        core.segment_sum(N, H, lv.rowptr, None, g0, ref)
    res = {}
    for name, f in (("fused backward", bwd(False)), ("fused backward + dP_d", bwd(True)),
                    ("segment_sum (dP_d)", seg)):
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record()
            f()
            b.record()
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)
        res[name] = ms[len(ms) // 2]
        print(f"N = {N}, E = {E}: {name:24s} {res[name]:.3f} ms (median of {args.reps}, HIP events)")
    bwd(True)()
    seg()
    torch.cuda.synchronize()
    nd = (dpd.view(torch.int16) != ref.view(torch.int16)).sum().item()
    print(f"dP_d elements differing from agn_segment_sum: {nd}")
    d = res["fused backward + dP_d"] - res["fused backward"]
    print(f"dP_d adds {d:.3f} ms to the fused launch; the segment_sum it replaces takes {res['segment_sum (dP_d)']:.3f} ms")


if __name__ == "__main__":
    main()
