"""Phase clocks of agn_edge_bwd_fused (diagnostic run, not the product path): one C3 level-0
MeshGraphNetLayer fwd+bwd with core.STAMPS set; prints the median cycles per phase per round."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
from aerognn import core  # noqa: E402
from aerognn.graph import Level  # noqa: E402
from aerognn.meshgen import ellipsoid  # noqa: E402
from models.mgnLayer import MeshGraphNetLayer  # noqa: E402

m = ellipsoid(1000, 1000)
ei = torch.from_numpy(m["edge_index"]).cuda()
N, E = m["x"].shape[0], ei.shape[1]
lv = Level.from_edge_index(ei, N)
torch.manual_seed(0)
layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).cuda()
x = torch.randn(N, 128, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
e = torch.randn(E, 128, device="cuda", dtype=torch.bfloat16).requires_grad_(True)
for it in range(3):
    core.STAMPS = torch.zeros(2 * 4 * 8 * 32, dtype=torch.int64, device="cuda") if it == 2 else None
    xo, eo = layer.forward_level(x, e, lv)
    (xo.float().sum() + eo.float().sum()).backward()
    torch.cuda.synchronize()
st = core.STAMPS.cpu().numpy().reshape(2, 4, 8, 32).astype(np.int64)
names = ["start"] + [f"L{L}:{k}" for L in (3, 2, 1) for k in ("dW", "chain", "barB", "drain", "barA")] + \
        ["s0:chain", "s0:stores", "s0:drain", "s0:bar"]
pts = [0] + [1 + 5 * (3 - L) + k for L in (3, 2, 1) for k in range(5)] + [16, 17, 18, 19]
d = np.diff(st[:, :, 1:7, pts], axis=-1)  # rounds 1..6 (skip the first)
med = np.median(d.reshape(-1, d.shape[-1]), axis=0)
for n, v in zip(names[1:], med):
    print(f"{n:10s} {v:8.0f}")
tot = np.median((st[:, :, 2:7, 0] - st[:, :, 1:6, 0]).reshape(-1))
print(f"round total {tot:.0f} cycles")
