"""Micro-benchmark of one MeshGraphNetLayer (EdgeBlockSum + NodeBlock, H=128) forward+backward
at the C3 fine level (1M nodes / 6M edges, bf16) — for counter profiling of the hot kernels
without the rest of the U-Net.  Usage: python tools/layer_micro.py [iters] [nu] [nv]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")

import torch  # noqa: E402

from aerognn.graph import Level  # noqa: E402
from aerognn.meshgen import ellipsoid  # noqa: E402
from models.mgnLayer import MeshGraphNetLayer  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    nu = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    nv = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    dev = torch.device("cuda", 0)
    m = ellipsoid(nu, nv, seed=0)
    ei = torch.from_numpy(m["edge_index"]).to(dev)
    N, E = m["x"].shape[0], ei.shape[1]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).to(dev)
    lv = Level.from_edge_index(ei, N)
    x = torch.randn(N, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
    e = torch.randn(E, 128, device=dev, dtype=torch.bfloat16, requires_grad=True)
    for i in range(iters + 1):
        if i == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        xo, eo = layer.forward_level(x, e, lv)
        (xo.float().square().sum() + eo.float().square().sum()).backward()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    print(f"N={N} E={E} layer fwd+bwd {dt * 1e3:.2f} ms  {E / dt / 1e6:.1f} M EU/s", flush=True)


if __name__ == "__main__":
    main()
