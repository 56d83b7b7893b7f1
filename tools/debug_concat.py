"""Diagnostics (GPU, not a test): the concat edge MLP layer's dx at C2 size, the product path
(agn_segment_sum2) against the two-segment-sum composition it replaced, and both against the
CPU oracle, with the worst nodes' degrees."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from aerognn import functions as F
    from aerognn import core
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    from oracle import refcpu as R
    nu, nv = int(os.environ.get("NU", "400")), int(os.environ.get("NV", "250"))
    m = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=0).items()}
    N, E = m["x"].shape[0], m["edge_index"].shape[1]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=False)
    g = torch.Generator(device="cpu").manual_seed(4)
    x = torch.randn(N, 128, generator=g)
    e = torch.randn(E, 128, generator=g)
    gxo = torch.randn(N, 128, generator=g)
    geo = torch.randn(E, 128, generator=g)
    p = {f"L.{k}": v.clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    cfg = R.cfg_from_kwargs(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                            do_concat_trick=False, aggregation="add")
    xr_in, er_in = x.clone().requires_grad_(True), e.clone().requires_grad_(True)
    xr, er = R.gmp_layer(p, "L", xr_in, er_in, m["edge_index"], cfg)
    torch.autograd.backward([xr, er], [gxo, geo])
    layer = layer.cuda()

    def run():
        xg, eg = x.cuda().requires_grad_(True), e.cuda().requires_grad_(True)
        xo, eo = layer(xg, eg, m["edge_index"].cuda())
        torch.autograd.backward([xo, eo], [gxo.cuda(), geo.cuda()])
        torch.cuda.synchronize()
        return xg.grad.cpu(), eg.grad.cpu()
    dx_new, de_new = run()
    orig = F.segment_sum2

    def old(n, h, base, a, b, out):
        ds = core.segment_sum(n, h, a[0], a[1], a[2], torch.empty(n, h, dtype=a[2].dtype, device=a[2].device))
        dd = core.segment_sum(n, h, b[0], b[1], b[2], torch.empty(n, h, dtype=a[2].dtype, device=a[2].device))
        out.copy_((base if base is not None else 0) + ds + dd)
        return out
    F.segment_sum2 = old
    dx_old, _ = run()
    F.segment_sum2 = orig
    ref = xr_in.grad
    deg_in = torch.bincount(m["edge_index"][1], minlength=N)
    deg_out = torch.bincount(m["edge_index"][0], minlength=N)
    for name, d in (("new", dx_new), ("old", dx_old)):
        err = (d - ref).abs().amax(1) / ref.abs().amax()
        w = torch.argsort(err, descending=True)[:8]
        print(f"{name}: rel-L2 {float((d - ref).norm() / ref.norm()):.2e}; worst nodes {w.tolist()} err "
              f"{[round(float(err[i]), 5) for i in w]} in-deg {deg_in[w].tolist()} out-deg {deg_out[w].tolist()}")
    print("de rel-L2", float((de_new - er_in.grad).norm() / er_in.grad.norm()))
    print("new vs old max abs", float((dx_new - dx_old).abs().max()))


if __name__ == "__main__":
    main()
