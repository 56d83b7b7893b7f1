"""Per-mesh hierarchy caches: the opt-in BiStridedMeshGraphNet cache and the
BSMS-GNN dataset wrapper return exactly what a rebuild returns, and invalidate on change."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
os.environ.setdefault("AEROGNN_MEMLOG", "0")
DEV = "cuda"


def _mesh(nu, nv, seed=0):
    from aerognn.meshgen import ellipsoid
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(DEV) for k, v in ellipsoid(nu, nv, seed=seed).items()}


def test_bsms_mgn_hierarchy_cache_bitwise():
    from models.bsms_mgn import BiStridedMeshGraphNet
    t = _mesh(60, 40)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, num_scales=3, do_concat_trick=True).to(DEV)
    ref = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).detach()
    model.cache_hierarchy(True)
    a = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).detach()
    b = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).detach()
    assert len(model._hcache) == 1
    assert torch.equal(a, ref) and torch.equal(b, ref)
    # a modified mesh (in place: version bump + new contents) is a different hierarchy
    t["pos"][:, 0] *= -1.0
    c = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).detach()
    assert len(model._hcache) == 2
    model.cache_hierarchy(False)
    d = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).detach()
    assert torch.equal(c, d)
    # gradients flow through cached hierarchies as well
    model.cache_hierarchy(True)
    model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"]).float().square().mean().backward()
    assert all(p.grad is not None for p in model.parameters())


def test_bsms_dataset_wrapper_caches():
    from models.bsms_dataset_wrapper import BSMSDataLoader, BSMSDatasetWrapper, prepare_bsms_data
    from models.bsms_mgn import MultiScaleGraphPreprocessor

    class S:
        pass
    samples = []
    for seed in range(3):
        m = _mesh(20, 12, seed)
        s = S()
        s.x, s.edge_index, s.pos = m["x"].cpu(), m["edge_index"].cpu(), m["pos"].cpu()
        s.num_nodes = s.x.shape[0]
        samples.append(s)
    ds = BSMSDatasetWrapper(samples, num_levels=2)
    assert len(ds) == 3
    d0 = ds[0]
    again = ds.get(0)
    assert again.multi_data is d0.multi_data  # cached object
    ref = MultiScaleGraphPreprocessor(2).create_multiscale_graph(type("D", (), {
        "edge_index": samples[0].edge_index.to(DEV), "pos": samples[0].pos.to(DEV),
        "num_nodes": samples[0].num_nodes})())
    for a, b in zip(d0.multi_data["edge_indices"], ref["edge_indices"]):
        assert torch.equal(a, b)
    assert d0.multi_data["num_nodes"] == ref["num_nodes"]
    seen = [d for d in BSMSDataLoader(prepare_bsms_data(samples, 2), batch_size=4)]
    assert len(seen) == 3 and all(hasattr(d, "multi_data") for d in seen)
