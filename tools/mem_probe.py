"""HBM probes for the access patterns of the edge kernels (C3 fine level, bf16, 256-B rows):
streaming copy, row gathers by receiver (CSC order, sequential), by sender (CSC order, local)
and by a random permutation. torch kernels, HIP-event timed: an upper reference for what the
memory system delivers on each pattern, not a product path."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]

import torch  # noqa: E402

from aerognn.graph import Level  # noqa: E402
from aerognn.meshgen import ellipsoid  # noqa: E402


def timeit(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    return ms, nbytes / (ms * 1e-3) / 1e9


def main():
    dev = torch.device("cuda", 0)
    m = ellipsoid(1000, 1000, seed=0)
    ei = torch.from_numpy(m["edge_index"]).to(dev)
    N, E = m["x"].shape[0], ei.shape[1]
    lv = Level.from_edge_index(ei, N)
    H = 128
    x = torch.randn(N, H, device=dev, dtype=torch.bfloat16)
    e = torch.randn(E, H, device=dev, dtype=torch.bfloat16)
    out = torch.empty_like(e)
    src, dst = lv.src.long(), lv.dst.long()
    rnd = torch.randint(0, N, (E,), device=dev)
    row = E * H * 2
    res = {}
    res["copy e (read+write)"] = timeit(lambda: out.copy_(e), 2 * row)
    res["gather x[dst] (CSC)"] = timeit(lambda: torch.index_select(x, 0, dst, out=out), 2 * row)
    res["gather x[src] (CSC)"] = timeit(lambda: torch.index_select(x, 0, src, out=out), 2 * row)
    res["gather x[random]"] = timeit(lambda: torch.index_select(x, 0, rnd, out=out), 2 * row)
    big = torch.empty(E, 2 * H, device=dev, dtype=torch.bfloat16)
    res["write-only e x2 (fill)"] = timeit(lambda: big.fill_(1.0), 2 * row)
    res["read-only sum e"] = timeit(lambda: e.sum(), row)
    for k, (ms, gbs) in res.items():
        print(f"{k:28s} {ms:8.3f} ms  {gbs:8.1f} GB/s")


if __name__ == "__main__":
    main()
