"""A/B micro-timing of the grouped-row kernels (agn_segment_sum, agn_gather_rows) at C3 level-0
size, across builds of libaerognn loaded side by side through ctypes.

  python tools/seg_micro.py LIB_A.so [LIB_B.so ...]

Graph: a 1000 x 1000 triangulated grid (6 neighbours per interior node, ~6M directed edges), in
CSC order (grouped by receiver) like a Level, with the sender-grouped permutation beside it.
Per library and kernel: ms per launch (HIP events on torch's current stream, which the calls use)
and whether the output is bitwise equal to the first library's.
"""
import ctypes
import sys

import numpy as np
import torch

AGN_BF16 = 1
dev = torch.device("cuda", 0)


def grid_graph(n=1000):
    ids = np.arange(n * n).reshape(n, n)
    src, dst = [], []
    for di, dj in ((0, 1), (1, 0), (1, 1)):
        a = ids[: n - di, : n - dj].ravel()
        b = ids[di:, dj:].ravel()
        src += [a, b]
        dst += [b, a]
    src, dst = np.concatenate(src), np.concatenate(dst)
    o = np.argsort(dst, kind="stable")
    src, dst = src[o], dst[o]
    N = n * n
    rowptr = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(dst, minlength=N), out=rowptr[1:])
    perm_src = np.argsort(src, kind="stable")
    rowptr_src = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(src, minlength=N), out=rowptr_src[1:])
    t = lambda a: torch.from_numpy(a.astype(np.int32)).to(dev)  # noqa: E731
    return N, len(src), t(src), t(dst), t(rowptr), t(perm_src), t(rowptr_src)


def timeit(f, it=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main(libs):
    N, E, src, dst, rowptr, perm_src, rowptr_src = grid_graph()
    H = 128
    torch.manual_seed(0)
    g0 = torch.randn(E, H, device=dev).to(torch.bfloat16)
    xn = torch.randn(N, H, device=dev).to(torch.bfloat16)
    addE = torch.randn(E, H, device=dev).to(torch.bfloat16)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    print(f"N={N} E={E} H={H} bf16", flush=True)
    ref = {}
    for path in libs:
        L = ctypes.CDLL(path)
        outs = {}
        cases = {
            "segsum_src": lambda o: L.agn_segment_sum(N, H, AGN_BF16, p(rowptr_src), p(perm_src), p(g0), H, p(o),
                                                      H, 0, st),
            "segsum_dst": lambda o: L.agn_segment_sum(N, H, AGN_BF16, p(rowptr), None, p(g0), H, p(o), H, 0, st),
            "segsum_dst_mean": lambda o: L.agn_segment_sum(N, H, AGN_BF16, p(rowptr), None, p(g0), H, p(o), H, 1,
                                                           st),
            "segsum2": lambda o: L.agn_segment_sum2(N, H, AGN_BF16, p(xn), H, p(rowptr_src), p(perm_src), p(g0), H,
                                                    p(rowptr), None, p(g0), H, p(o), H, st),
            "gather_E_by_dst": lambda o: L.agn_gather_rows(E, H, AGN_BF16, p(dst), p(xn), H, None, None, 0, p(o), H,
                                                           st),
            "gather_E_perm_add": lambda o: L.agn_gather_rows(E, H, AGN_BF16, p(perm_src), p(g0), H, None, p(addE), H,
                                                             p(o), H, st),
            "gather_N_mean": lambda o: L.agn_gather_rows(N, H, AGN_BF16, None, p(xn), H, p(rowptr), None, 0, p(o), H,
                                                         st),
        }
        for name, f in cases.items():
            rows = E if name.startswith("gather_E") else N
            o = torch.empty(rows, H, dtype=torch.bfloat16, device=dev)
            rc = f(o)
            assert rc == 0, (name, rc)
            ms = timeit(lambda: f(o))
            same = None
            if name in ref:
                same = bool(torch.equal(ref[name].view(torch.int16), o.view(torch.int16)))
            else:
                ref[name] = o
            print(f"{path.split('/')[-1]:28s} {name:18s} {ms * 1e3:9.1f} us  bitwise_vs_first={same}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
