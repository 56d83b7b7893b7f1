"""Micro-timing of the fused path's dW_e launch (agn_wgrad: dW_e = G0^T e over the C3 level-0
edges, both row-major bf16 [E,128]) and of a node-side batch (N rows: the node MLP's four Linears
and the projection, tiled / row-major as the training step passes them). Prints ms per launch and
the operator-I/O rate (G and X read once)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
import torch  # noqa: E402

from aerognn.core import WGrad  # noqa: E402

E = int(sys.argv[1]) if len(sys.argv) > 1 else 5996000
dev = torch.device("cuda", 0)
torch.manual_seed(0)
bf = torch.bfloat16
g0 = torch.randn(E, 128, dtype=bf, device=dev) * 0.01
e = torch.randn(E, 128, dtype=bf, device=dev)
dwe = torch.empty(128, 128, dtype=torch.float32, device=dev)


def run():
    wg = WGrad()
    wg.add(g0, e, dwe)
    wg.run()


for _ in range(3):
    run()
torch.cuda.synchronize()
n = 10
t = time.perf_counter()
for _ in range(n):
    run()
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / n
by = 2 * E * 128 * 2
print(f"dW_e over E = {E}: {1e3 * dt:.3f} ms per launch, {by / dt / 1e9:.0f} GB/s of G + X")
