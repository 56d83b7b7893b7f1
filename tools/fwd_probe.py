"""What bounds the inference edge forward (diagnostic, not the product path): one C3 level-0 sized
layer (1M nodes / ~6M edges, ellipsoid mesh in CSC order), agn_edge_forward (16-row tiles) and
agn_edge_forward32 (32-row tiles) timed with the real sender ids, with the senders replaced by the
receivers (both projection gathers walk CSC order: L2-friendly), and with every id 0 (the gathers
hit one row: the chain's compute and the e / e' streams alone). HIP events, median of --reps.

Usage (GPU): python tools/fwd_probe.py [--nu 1000] [--reps 7]
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
    ap.add_argument("--real-only", action="store_true", help="only the real ids (counter passes)")
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
    spec = layer.spec()
    spec.pack.update(dt, dev)
    es = spec.edge
    P = torch.empty(N, 2 * H, dtype=dt, device=dev)
    core.proj_forward(N, x, spec.pack["proj"], spec.pack["proj_b"], P)
    out = torch.empty_like(e)
    zeros = torch.zeros_like(lv.dst)
    cases = (("real ids", lv.src, lv.dst), ("src := dst", lv.dst, lv.dst), ("all ids 0", zeros, zeros))
    for ids_name, src, dst in cases[:1] if args.real_only else cases:
        for kname in ("edge32 (32-row)",):
            def f():
                core.edge_forward(rows=E, wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), e=e, proj=P, src=src, dst=dst,
                                  out=out)
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
            t = ms[len(ms) // 2]
            print(f"N = {N}, E = {E}: {ids_name:11s} {kname:16s} {t * 1e3:8.1f} us  {E / t / 1e3:8.1f} M edges/s", flush=True)


if __name__ == "__main__":
    main()
