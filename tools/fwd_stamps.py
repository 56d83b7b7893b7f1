"""Phase clocks of the resident edge forward (mlp_fwd_res_kernel; diagnostics, GPU) on a
C5-sized level-0 layer (5M nodes / 30M edges, forward only, no saves) and a C3-sized one.

Usage: AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_stamps.so python tools/fwd_stamps.py
"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

PH = ["P gather + acc init", "e load + pack", "layer 0 gemm", "relu+bias L1", "gemm L1", "relu+bias L2",
      "gemm L2", "relu+bias L3", "gemm L3", "LN stats", "epilogue (LN, residual, pack)", "e' staged store"]


def run(nu, nv):
    from aerognn import core, _lib as L
    from aerognn.graph import Level
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    m = ellipsoid(nu, nv, seed=0)
    ei = torch.from_numpy(np.ascontiguousarray(m["edge_index"])).cuda()
    N, E, H = m["x"].shape[0], ei.shape[1], 128
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).cuda()
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    dt = torch.bfloat16
    x = torch.randn(N, H, generator=g).to("cuda", dt)
    e = torch.randn(E, H, generator=g).to("cuda", dt)
    spec = layer.spec()
    spec.pack.update(dt, "cuda")
    es = spec.edge
    P = torch.empty(N, 2 * H, dtype=dt, device="cuda")
    core.proj_forward(N, x, spec.pack["proj"], spec.pack["proj_b"], P)
    out = torch.empty_like(e)

    def fwd():
        core.mlp_forward(rows=E, dtype=dt, hidden=H, nlin=es.nlin, out_dim=H,
                         segs=[(L.SEG_PLAIN, H, e.stride(0), e, None, None)], wpk=es.wpk(), bias=es.biases(),
                         ln=es.lnp(), proj=P, src=lv.src, dst=lv.dst, resid=e, out=out)
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        fwd()
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t) / 5
    print(f"N={N} E={E}: {ms:.3f} ms per launch, {E * 520 / ms / 1e9:.2f} TB/s of 520 B/edge")
    st = torch.zeros(8 * 8 * 16, dtype=torch.int64, device="cuda")
    lib = L.lib()
    if lib.agn_debug_fwd_stamps(C.c_void_p(st.data_ptr())) != 0:
        raise SystemExit("stamps library required")
    fwd()
    torch.cuda.synchronize()
    lib.agn_debug_fwd_stamps(C.c_void_p(0))
    s = st.cpu().numpy().reshape(8, 8, 16).astype(np.int64)
    d = np.diff(s[:, 1:8, :13], axis=2)  # waves x tiles 1..7 x 12 phases
    per_tile = (s[:, 2:8, 0] - s[:, 1:7, 0]).mean()
    print(f"  cycles per tile per wave {per_tile:.0f} (2 waves share a SIMD)")
    print("  " + ", ".join(f"{p} {v:.0f}" for p, v in zip(PH, d.mean((0, 1)))))


if __name__ == "__main__":
    run(2500, 2000)
    run(1000, 1000)
