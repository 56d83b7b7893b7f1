"""Micro-timing of the edge encoder's weight-gradient launch (C3 level-0 rows) and its parts.

The encoder's first Linear reads edge_attr through the level-0 permutation, so its dW block uses
agn_wgrad's gathered operand (xidx, K = 4); the two hidden Linears are plain [E,128] x [E,128].
Prints ms per launch for: all three in one launch, the gathered one alone, the two plain ones alone.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
import torch  # noqa: E402

from aerognn.core import WGrad, tiled_empty  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 5996000
dev = torch.device("cuda", 0)
torch.manual_seed(0)
bf = torch.bfloat16


def tiled(rows, w):
    t = tiled_empty(rows, w, bf, dev)
    t.normal_()
    return t


G = [tiled(E, 128) for _ in range(3)]
A = [tiled(E, 128) for _ in range(2)]
ea = torch.randn(E, 4, dtype=bf, device=dev)
idx = torch.randperm(E, device=dev).to(torch.int32)
dw0 = torch.empty(128, 4, dtype=torch.float32, device=dev)
db0 = torch.empty(128, dtype=torch.float32, device=dev)
dw = [torch.empty(128, 128, dtype=torch.float32, device=dev) for _ in range(2)]
db = [torch.empty(128, dtype=torch.float32, device=dev) for _ in range(2)]


def run(parts):
    wg = WGrad()
    if 0 in parts:
        wg.add(G[0], ea, dw0, db0, xidx=idx)
    for j in (1, 2):
        if j in parts:
            wg.add(G[j], A[j - 1], dw[j - 1], db[j - 1])
    wg.run()


for name, parts in (("all three (one launch)", (0, 1, 2)), ("gathered W0 alone", (0,)), ("W1+W2", (1, 2)),
                    ("W0 ungathered", None)):
    if parts is None:
        def f():
            wg = WGrad()
            wg.add(G[0], ea, dw0, db0)
            wg.run()
    else:
        def f(parts=parts):
            run(parts)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        f()
    e.record()
    torch.cuda.synchronize()
    print(f"{name:28s} {s.elapsed_time(e) / 10:8.3f} ms", flush=True)
