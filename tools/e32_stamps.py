"""Phase clocks of the 32-row edge forward (edge32_fwd_kernel; diagnostics, GPU) on a C3-sized
level-0 layer (1M nodes / 6M edges, ellipsoid mesh in CSC order), with the real sender ids and with
every id 0. Needs a library built with -DAGN_E32_STAMPS:

  AEROGNN_LIB=aero-gnn_amd/aerognn/libaerognn_e32st.so python tools/e32_stamps.py

Per phase: mean cycles per tile per wave (12 waves per CU, three per SIMD), from the waves of
block 0 over tiles 2..15; the in-kernel clock from s_memtime against s_memrealtime (100 MHz).
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402

PH = ["loads + row sum", "gemm L0", "relu+bias+gemm L1", "relu+bias+gemm L2", "relu+bias+gemm L3", "LN stats",
      "epilogue + stores", "to next tile"]


def main(nu=1000):
    from aerognn import core, _lib as L
    from aerognn.graph import Level
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    m = ellipsoid(nu, nu, seed=0)
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
    lib = L.lib()
    zeros = torch.zeros_like(lv.dst)
    for name, src, dst in (("real ids", lv.src, lv.dst), ("all ids 0", zeros, zeros)):
        def fwd():
            core.edge_forward(rows=E, wpk=es.wpk(), bias=es.biases(), ln=es.lnp(), e=e, proj=P, src=src, dst=dst,
                              out=out)
        for _ in range(3):
            fwd()
        torch.cuda.synchronize()
        st = torch.zeros(16 * 16 * 16, dtype=torch.int64, device="cuda")
        if lib.agn_debug_e32_stamps(C.c_void_p(st.data_ptr())) != 0:
            raise SystemExit("stamps library required")
        fwd()
        torch.cuda.synchronize()
        lib.agn_debug_e32_stamps(C.c_void_p(0))
        s = st.cpu().numpy().reshape(16, 16, 16).astype(np.int64)[:12]
        t0, rt = s[:, :, 0], s[:, :, 15]
        ok = (t0[:, 2:] > 0).all()
        per_tile = (t0[:, 3:16] - t0[:, 2:15]).mean()
        clock = (t0[:, 15] - t0[:, 2]).sum() / (rt[:, 15] - rt[:, 2]).sum() * 0.1
        ph = np.concatenate([np.diff(s[:, 2:15, :8], axis=2), (t0[:, 3:16] - s[:, 2:15, 7])[:, :, None]], axis=2)
        print(f"N={N} E={E} {name}: {per_tile:.0f} cycles per tile per wave (3 waves per SIMD: "
              f"{per_tile / 3:.0f} per tile per SIMD), in-kernel clock {clock:.2f} GHz{'' if ok else ' (incomplete)'}")
        print("  " + ", ".join(f"{p} {v:.0f}" for p, v in zip(PH, ph.mean((0, 1)))))


if __name__ == "__main__":
    main()
