"""Phase clocks of agn_edge_backward (diagnostic run, not the product path): one C3 level-0 sized
layer (1M nodes / ~6M edges), timed with the product library and then once with the
-DAGN_E16_STAMPS library (AEROGNN_LIB), s_memtime per phase of the chain waves of blocks 0 and 128
(8 tiles each) and the dW waves' idle share.

Usage (GPU): python tools/e16_stamps.py [--lib aero-gnn_amd/aerognn/libaerognn_stamps.so]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")

PHASES = ["loads + P sum", "forward (4 GEMMs)", "LN stats + S", "LN backward", "recompute a2, a3",
          "wait slot L3", "write L3", "chain L3", "wait slot L2", "write L2", "chain L2", "wait slot L1",
          "write L1", "chain L1", "step 0 (G0 W_e, de)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nu", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stamps", action="store_true", help="AEROGNN_LIB is a stamps build: print phase clocks")
    ap.add_argument("--save", default=None, help="save the raw stamps [2][16][8][16] (.npy)")
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
    out = torch.empty_like(e)

    def fwd():
        core.edge_forward(rows=E, wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), e=e, proj=P, src=lv.src,
                          dst=lv.dst, out=out)

    def bwd():
        return core.edge_bwd_fused(rows=E, wpk=es.wpk(), bias=es.biases(), ln_g=es.lnp()[0], e=e, proj=P,
                                   src=lv.src, dst=lv.dst, g=ge, g2=dagg, de=de, g0=g0, e16=True)
    for name, f in (("forward", fwd), ("backward", bwd)):
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
        print(f"E = {E}: edge16 {name} {ms[len(ms) // 2]:.3f} ms per launch (median of {args.reps}, HIP events)")
    if not args.stamps:
        return
    core.STAMPS = torch.zeros(2 * 16 * 8 * 16, dtype=torch.int64, device=dev)
    bwd()
    torch.cuda.synchronize()
    st = core.STAMPS.cpu().numpy().astype(np.int64).reshape(2, 16, 8, 16)
    core.STAMPS = None
    if args.save:
        np.save(args.save, st)
    ch = st[:, :8]  # chain waves
    d = np.diff(ch, axis=-1)  # [2, 8, 8, 15] phase durations
    tile = ch[..., 15] - ch[..., 0]
    print(f"chain waves: cycles per 16-edge tile: median {np.median(tile):.0f}, mean {tile.mean():.0f}")
    for k, name in enumerate(PHASES):
        v = d[..., k]
        print(f"  {name:22s} median {np.median(v):7.0f}  mean {v.mean():7.0f}  max {v.max():7.0f}")
    # tile-to-tile gaps (loop overhead, partial rounds)
    gap = ch[..., 1:, 0] - ch[..., :-1, 15]
    print(f"  {'between tiles':22s} median {np.median(gap):7.0f}")
    dw = st[:, 8:, 0, :3]
    for s in range(2):
        for w in range(8):
            waited, tot, n = dw[s, w]
            if tot:
                print(f"  block {0 if s == 0 else 128} dW wave {w}: idle {waited / tot:.2f} of {tot} cycles, {n} items/layer")


if __name__ == "__main__":
    main()
