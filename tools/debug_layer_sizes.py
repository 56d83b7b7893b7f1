"""Diagnostics (GPU, not a test): one fp32 MeshGraphNetLayer forward + backward against the CPU
oracle's autograd over mesh sizes, concat and sum-trick edge blocks: where do gradients drift?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def one(nu, nv, trick):
    from aerognn.meshgen import ellipsoid
    from models.mgnLayer import MeshGraphNetLayer
    from oracle import refcpu as R
    m = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=0).items()}
    N, E = m["x"].shape[0], m["edge_index"].shape[1]
    torch.manual_seed(0)
    layer = MeshGraphNetLayer(128, 128, 128, 2, 2, do_concat_trick=trick)
    g = torch.Generator(device="cpu").manual_seed(4)
    x, e = torch.randn(N, 128, generator=g), torch.randn(E, 128, generator=g)
    gxo, geo = torch.randn(N, 128, generator=g), torch.randn(E, 128, generator=g)
    p = {f"L.{k}": v.clone().requires_grad_(True) for k, v in layer.state_dict().items()}
    cfg = R.cfg_from_kwargs(num_hidden_layers_node_processor=2, num_hidden_layers_edge_processor=2,
                            do_concat_trick=trick, aggregation="add")
    xr_in, er_in = x.clone().requires_grad_(True), e.clone().requires_grad_(True)
    xr, er = R.gmp_layer(p, "L", xr_in, er_in, m["edge_index"], cfg)
    torch.autograd.backward([xr, er], [gxo, geo])
    layer = layer.cuda()
    xg, eg = x.cuda().requires_grad_(True), e.cuda().requires_grad_(True)
    xo, eo = layer(xg, eg, m["edge_index"].cuda())
    torch.autograd.backward([xo, eo], [gxo.cuda(), geo.cuda()])
    torch.cuda.synchronize()
    pg = sorted(((rel(q.grad.cpu(), p[f"L.{n}"].grad), n) for n, q in layer.named_parameters()), reverse=True)
    print(f"{'sum' if trick else 'cat'} N={N} E={E}: x' {rel(xo.detach().cpu(), xr.detach()):.1e} "
          f"e' {rel(eo.detach().cpu(), er.detach()):.1e} dx {rel(xg.grad.cpu(), xr_in.grad):.1e} "
          f"de {rel(eg.grad.cpu(), er_in.grad):.1e} worst param {pg[0][0]:.1e} ({pg[0][1]}) "
          f"2nd {pg[1][0]:.1e} ({pg[1][1]})", flush=True)


if __name__ == "__main__":
    for trick in (False, True):
        for nu, nv in ((24, 16), (60, 40), (120, 80), (150, 110), (250, 200), (400, 250)):
            one(nu, nv, trick)
