"""One concat edge-MLP layer (do_concat_trick=False, mgnLayer.py:10-49), fp32 at C2 size, forward
and backward, for a rocprofv3 kernel trace: every kernel the layer launches should be a
libaerognn kernel (no torch / aten kernels). Inputs are built and copied before the marked region.
Usage (GPU): rocprofv3 --kernel-trace --stats -d DIR -o concat -- python tools/concat_trace.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    m = ellipsoid(400, 250, seed=0)
    ei = torch.from_numpy(np.ascontiguousarray(m["edge_index"])).cuda()
    N, E = m["x"].shape[0], ei.shape[1]
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(N, 128, generator=g).cuda().requires_grad_(True)
    e = torch.randn(E, 128, generator=g).cuda().requires_grad_(True)
    gx, ge = torch.randn(N, 128, generator=g).cuda(), torch.randn(E, 128, generator=g).cuda()
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=False).cuda()
    torch.cuda.synchronize()
    print("== layer start ==", flush=True)
    xo, eo = layer(x, e, ei)
    torch.autograd.backward([xo, eo], [gx, ge])
    torch.cuda.synchronize()
    print("== layer end ==", flush=True)


if __name__ == "__main__":
    main()
