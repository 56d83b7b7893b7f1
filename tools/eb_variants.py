"""Same-box timing of the fused edge backward's variants (round 6) on one C3 level-0 sized layer
(1M nodes / ~6M edges, ellipsoid mesh in CSC order): the recompute started from the forward's a1 /
LayerNorm statistics or from e and the projection rows, and a2 parked in the scratch or
recomputed; plus the edge forward with and without its training saves. HIP events around each
launch, medians over REPS launches, the variants interleaved so box drift hits them alike.

Usage (GPU): python tools/eb_variants.py [--reps 20]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--nu", type=int, default=1000)
    ap.add_argument("--only", default=None, help="substring filter on the case names")
    args = ap.parse_args()
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
    out = torch.empty_like(e)
    a1 = core.tiled_empty(E, H, dt, e.device)
    st = torch.empty(E, 2, dtype=torch.float32, device=dev)
    de = torch.empty_like(e)
    g0 = torch.empty(E, H, dtype=dt, device=dev)
    dpd = torch.empty(N, H, dtype=dt, device=dev)

    def fwd(save):
        return lambda: core.edge_forward(rows=E, wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), e=e, proj=P,
                                         src=lv.src, dst=lv.dst, out=out, a1=a1 if save else None,
                                         stats=st if save else None)

    def bwd(saved, scr):
        return lambda: core.edge_bwd_fused(rows=E, wpk=es.wpk(), wtpk0=es.wtpk()[0], bias=es.biases(), ln_g=es.lnp()[0], e=e, proj=P,
                                           src=lv.src, dst=lv.dst, g=ge, g2=dagg, de=de, g0=g0,
                                           a1=a1 if saved else None, stats=st if saved else None, scratch=scr)
    cases = {"fwd (no saves)": fwd(False), "fwd + a1/stats saves": fwd(True)}
    for saved in (True, False):
        for scr in (True, False):
            cases[f"bwd saved={int(saved)} scratch={int(scr)}"] = bwd(saved, scr)
    cases["segment_sum (dP_d)"] = lambda: core.segment_sum(N, H, lv.rowptr, None, g0, dpd)
    if args.only:
        cases = {k: v for k, v in cases.items() if args.only in k}
    fwd(True)()
    for f in cases.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    for _ in range(args.reps):
        for k, f in cases.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            times[k].append((a, b))
    torch.cuda.synchronize()
    print(f"N = {N}, E = {E}, {args.reps} launches each (median / min ms, HIP events incl. the backward's slab "
          "reduce)")
    for k, evs in times.items():
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        print(f"  {k:32s} {ms[len(ms) // 2]:8.3f} {ms[0]:8.3f}", flush=True)


if __name__ == "__main__":
    main()
