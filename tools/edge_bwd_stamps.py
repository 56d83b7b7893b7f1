"""Phase clocks of agn_edge_bwd_fused (diagnostic run, not the product path): one C3 level-0
sized layer (1M nodes / ~6M edges), the -DAGN_EB_STAMPS library (AEROGNN_LIB), s_memtime per
phase of the chain waves of blocks 0 and 128 (8 tiles each) and the dW waves' wait share.

Usage (GPU): AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so python tools/edge_bwd_stamps.py
SAVED=1 (default): the recompute starts from the forward's a1 / statistics; SCR=1: a2 through the
scratch (default 0: a2 recomputed from a1; a3 stays in registers from the forward recompute).
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ["ids+loads", "forward", "LN stats+bwd", "recompute a2", "produce L3", "chain L3", "produce L2",
          "chain L2", "produce L1", "chain L1", "step 0 (de, G0)"]


def main():
    from aerognn import core
    from aerognn.graph import Level
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    dev = "cuda"
    nu = int(os.environ.get("NU", "1000"))
    m = ellipsoid(nu, nu, seed=0)
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

    saved = os.environ.get("SAVED", "1") == "1"
    scr = os.environ.get("SCR", "0") == "1"
    a1 = lnst = None
    if saved:
        a1 = core.tiled_empty(E, H, dt, e.device)
        lnst = torch.empty(E, 2, dtype=torch.float32, device=dev)
        core.edge_forward(rows=E, wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), e=e, proj=P, src=lv.src, dst=lv.dst,
                          out=torch.empty_like(e), a1=a1, stats=lnst)
    print(f"saved a1 / statistics: {saved}; a2 scratch: {scr}")

    def run():
        return core.edge_bwd_fused(rows=E, wpk=es.wpk(), wtpk0=es.wtpk()[0], bias=es.biases(), ln_g=es.lnp()[0], e=e, proj=P,
                                   src=lv.src, dst=lv.dst, g=ge, g2=dagg, de=de, g0=g0,
                                   a1=a1, stats=lnst, scratch=scr)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    print(f"E = {E}: {1e3 * (time.perf_counter() - t) / 5:.3f} ms per launch (incl. the slab reduce)")
    core.STAMPS = torch.zeros(4096, dtype=torch.int64, device=dev)
    run()
    torch.cuda.synchronize()
    allst = core.STAMPS.cpu().numpy().astype(np.int64)
    st = allst[:2048].reshape(2, 8, 8, 16)
    core.STAMPS = None
    # item timeline of block 0, rounds 1 and 2 (items 24..71): produce enter / slot free / flagged,
    # and per dW wave poll start / detect / released
    dwi = allst[2048:2048 + 576].reshape(4, 48, 3)
    chi = allst[2048 + 576:2048 + 576 + 144].reshape(4, 2, 6, 3)
    t0 = chi[:, 0, 0, 0].min()
    print("items  chain  enter  slotfree  flagged | dW detect (d0..d3, both items) | dW released | slot-wait  write  detect  read")
    for r in (1, 2):
        for li in range(3):
            for c in range(4):
                n = 24 * r + (12 if c >= 2 else 0) + 4 * li + 2 * (c & 1)  # edge_bwd.hip item order
                pe, pf, pg = chi[c, r - 1, 2 * li] - t0
                det = dwi[:, n - 24:n - 22, 1] - t0
                rel = dwi[:, n - 24:n - 22, 2] - t0
                print(f"{n:3d},{n + 1:3d} c{c} L{3 - li} {pe:7d} {pf:7d} {pg:7d} | " + " ".join(f"{x:7d}" for x in det.max(1)) +
                      " | " + " ".join(f"{x:7d}" for x in rel.max(1)) +
                      f" | {pf - pe:6d} {pg - pf:6d} {det[:, 0].max() - pg:6d} {rel[:, 1].max() - det[:, 0].max():6d}")
    for sel in range(2):
        print(f"block {0 if sel == 0 else 128}:")
        tot = np.zeros(len(PHASES))
        for w in range(4):
            s = st[sel, w]
            d = np.diff(s[1:8, :12], axis=1)  # tiles 1..7, phases 0..11
            tot += d.mean(0)
            per_tile = (s[2:8, 0] - s[1:7, 0]).mean()
            print(f"  chain wave {w}: cycles/tile {per_tile:9.0f}   " +
                  " ".join(f"{x:6.0f}" for x in d.mean(0)))
        print("  phases (mean over waves): " + ", ".join(f"{p} {v / 4:.0f}" for p, v in zip(PHASES, tot)))
        for dwv in range(4):
            s = st[sel, 4 + dwv]
            print(f"  dW wave {dwv}: waited {s[0, 0]} of {s[0, 1]} cycles ({s[0, 0] / max(s[0, 1], 1):.2f}), items {s[0, 2]}"
                  )


if __name__ == "__main__":
    main()
