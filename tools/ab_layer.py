"""A/B of one bf16 sum-trick MeshGraphNetLayer step at E = 98,400 (the fused-vs-split test's case)
for both edge-backward paths. Usage:
  AEROGNN_LIB=<lib.so> python tools/ab_layer.py save OUT.pt
  python tools/ab_layer.py cmp A.pt B.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd"), os.path.join(ROOT, "tests")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402


def run():
    from aerognn.graph import Level
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    m = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(150, 110, seed=0).items()}
    ei = m["edge_index"].cuda()
    N = m["x"].shape[0]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=True).cuda()
    lv = Level.from_edge_index(ei, N)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(N, 128, generator=g).cuda().bfloat16()
    e = torch.randn(ei.shape[1], 128, generator=g).cuda().bfloat16()
    out = {}
    for path in ("1", "0"):
        os.environ["AEROGNN_FUSED_EDGE_BWD"] = path
        xg, eg = x.clone().requires_grad_(True), e.clone().requires_grad_(True)
        layer.zero_grad()
        xo, eo = layer.forward_level(xg, eg, lv)
        (xo.float().square().sum() + 0.5 * eo.float().square().sum()).backward()
        torch.cuda.synchronize()
        tag = "fused" if path == "1" else "split"
        out.update({f"{tag}/x'": xo.detach().cpu(), f"{tag}/e'": eo.detach().cpu(), f"{tag}/dx": xg.grad.cpu(),
                    f"{tag}/de": eg.grad.cpu()})
        out.update({f"{tag}/g:{n}": p.grad.cpu() for n, p in layer.named_parameters()})
    return out


def main():
    if sys.argv[1] == "save":
        torch.save(run(), sys.argv[2])
        return
    a = torch.load(sys.argv[2], weights_only=True)
    b = torch.load(sys.argv[3], weights_only=True)
    for k in a:
        same = torch.equal(a[k], b[k])
        if not same:
            d = a[k].double() - b[k].double()
            print(f"  {k}: DIFF rel-L2 {float(d.norm() / b[k].double().norm()):.3e}")
    print(sum(torch.equal(a[k], b[k]) for k in a), "of", len(a), "equal")
    for side in (a, b):
        for k in ("x'", "e'", "dx", "de"):
            print("fused vs split", k, torch.equal(side["fused/" + k], side["split/" + k]))


if __name__ == "__main__":
    main()
