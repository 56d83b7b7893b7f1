"""Device data preparation vs the reference's formulas (oracle/refcpu.py,
restated from dataset.py:39-106 / :358-409 and PyG collate), and the fused edge-encoder gather.

* edge features: the displacement columns are bit-exact; the length column (torch.norm on the
  CPU) within 1 ulp (our fma order is torch's scalar order; its vectorised path regroups);
* normalisation statistics (torch.std_mean, unbiased) within 1e-6 relative; (v - mean) / std and
  its inverse bit-exact given the same statistics;
* collate: edge_index offsets and `batch` bit-exact vs aerognn.meshgen.collate (PyG semantics);
* MLP.forward_rows(x, perm) == MLP.forward(x[perm]) bitwise (forward and gradients).
"""
import os
import types

import numpy as np
import pytest
import torch

from golden_util import rel_l2

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"


def _mesh(nu, nv, seed=0):
    from aerognn.meshgen import ellipsoid
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in ellipsoid(nu, nv, seed=seed).items()}


def test_edge_features_and_perm():
    from aerognn import data as D
    from aerognn.graph import Level
    from oracle import refcpu as R
    m = _mesh(300, 200, seed=3)
    pos, ei = m["pos"], m["edge_index"]
    ref = R.compute_edge_attr(pos, ei)
    got = D.compute_edge_attr(pos=pos.to(DEV), edge_index=ei.to(DEV)).cpu()
    assert torch.equal(got[:, :3], ref[:, :3])
    ulp = (got[:, 3].view(torch.int32) - ref[:, 3].view(torch.int32)).abs()
    print(f"length column: {float((ulp > 0).float().mean()):.2e} of rows 1 ulp off, max {int(ulp.max())} ulp")
    assert int(ulp.max()) <= 1
    lv = Level.from_edge_index(ei.to(DEV), pos.shape[0])
    gp = D.compute_edge_attr(pos=pos.to(DEV), edge_index=ei.to(DEV), perm=lv.perm).cpu()
    assert torch.equal(gp, got[lv.perm.cpu()])


def test_normalization_stats_and_apply():
    from aerognn import data as D
    from oracle import refcpu as R
    samples = []
    for s in range(3):
        m = _mesh(60 + 10 * s, 40, seed=s)
        d = types.SimpleNamespace(x=m["x"].to(DEV), edge_attr=m["edge_attr"].to(DEV), y=m["y"].to(DEV))
        samples.append(d)
    ref = R.compute_normalization_stats([d.x.cpu() for d in samples], [d.edge_attr.cpu() for d in samples],
                                        [d.y.cpu() for d in samples])
    st = D.compute_normalization_stats(samples)
    for k in ref:  # means near 0 (unit-normal components): compare in units of the column's std
        scale = ref[k.replace("mean", "std")]
        err = float(((st[k].cpu() - ref[k]).abs() / scale).max())
        print(f"{k}: max |ours - torch| / std = {err:.2e}")
        assert err <= 2e-6, (k, err)
    raw = [(d.x.cpu(), d.edge_attr.cpu(), d.y.cpu()) for d in samples]
    D.normalize_data(samples, {k: v.to(DEV) for k, v in ref.items()})  # the reference's statistics: bit-exact
    for d, (x, e, y) in zip(samples, raw):
        assert torch.equal(d.x.cpu(), R.normalize(x, ref["node_mean"], ref["node_std"]))
        assert torch.equal(d.edge_attr.cpu(), R.normalize(e, ref["edge_mean"], ref["edge_std"]))
        assert torch.equal(d.y.cpu(), R.normalize(y, ref["target_mean"], ref["target_std"]))
    back = D.denormalize_predictions(samples[0].y, {k: v.to(DEV) for k, v in ref.items()}).cpu()
    with pytest.raises(RuntimeError):  # host statistics are refused, not dereferenced by the kernel
        D.denormalize_predictions(samples[0].y, ref)
    assert torch.equal(back, samples[0].y.cpu() * ref["target_std"] + ref["target_mean"])


def test_device_collate_matches_pyg_semantics():
    from aerognn import data as D
    from aerognn.meshgen import collate, ellipsoid
    ms = [ellipsoid(20 + 3 * s, 12, seed=s) for s in range(5)]
    ref = collate(ms)
    samples = [types.SimpleNamespace(**{k: torch.from_numpy(np.ascontiguousarray(m[k])).to(DEV)
                                        for k in ("x", "edge_attr", "y", "pos", "edge_index")}) for m in ms]
    out = D.collate(samples)
    assert torch.equal(out.edge_index.cpu(), torch.from_numpy(ref["edge_index"]))
    assert torch.equal(out.batch.cpu(), torch.from_numpy(ref["batch"]))
    for k in ("x", "edge_attr", "y", "pos"):
        assert torch.equal(getattr(out, k).cpu(), torch.from_numpy(ref[k]))
    assert out.num_graphs == 5 and out.num_nodes == ref["x"].shape[0]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_edge_encoder_fused_gather(dtype):
    """The edge encoder reads the caller's edge rows through the level permutation inside its
    first layer (no permuted copy): identical to encoding the gathered copy."""
    from models.mlp import MLP
    g = torch.Generator().manual_seed(0)
    E = 70_000
    ea = torch.randn(E, 4, generator=g).to(DEV, dtype)
    perm = torch.randperm(E, generator=g).to(DEV)
    torch.manual_seed(0)
    enc = MLP(4, 128, 128, num_hidden_layers=2).to(DEV)
    gy = torch.randn(E, 128, generator=g).to(DEV, dtype)
    outs = []
    for fused in (True, False):
        enc.zero_grad()
        x = ea.clone().requires_grad_(True)
        y = enc.forward_rows(x, perm) if fused else enc(x[perm])
        y.backward(gy)
        torch.cuda.synchronize()
        outs.append((y.detach(), x.grad.clone(), [p.grad.clone() for p in enc.parameters()]))
    assert torch.equal(outs[0][0], outs[1][0])
    assert rel_l2(outs[0][1].float(), outs[1][1].double()) <= (1e-6 if dtype == torch.float32 else 1e-2)
    for a, b in zip(outs[0][2], outs[1][2]):
        assert rel_l2(a.float(), b.double()) <= 1e-5
