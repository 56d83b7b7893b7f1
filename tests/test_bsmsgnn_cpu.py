"""CPU tests of the stale BSMS-GNN design: the oracle restatement
(oracle/bsmsgnn.py) pinned on hand-computed cases — parity with the reference itself is
UNPINNED (its bytecode cannot be executed here) — and the drop-in modules' construction,
state_dict schema and error behaviour."""
import pytest
import torch

from oracle import bsmsgnn as O


def _ei(pairs):
    return torch.tensor(pairs, dtype=torch.long).t().contiguous()


def test_bfs_path_and_unreachable():
    # 0 -> 1 -> 2 -> 3, 4 isolated, 5 -> 0 (5 unreachable from 0: edges are directed src -> dst)
    ei = _ei([(0, 1), (1, 2), (2, 3), (5, 0)])
    d = O.bfs_distance(ei, 6, 0)
    assert d.tolist() == [0, 1, 2, 3, -1, -1]


def test_bfs_shortest_hops_on_cycle():
    n = 7
    pairs = [(i, (i + 1) % n) for i in range(n)] + [((i + 1) % n, i) for i in range(n)]
    d = O.bfs_distance(_ei(pairs), n, 0)
    assert d.tolist() == [0, 1, 2, 3, 3, 2, 1]


def test_select_even_levels_and_fallback():
    # undirected path 0-1-2-3-4: seed = max out-degree (node 1, first of ties 1,2,3)
    pairs = [(0, 1), (1, 0), (1, 2), (2, 1), (2, 3), (3, 2), (3, 4), (4, 3)]
    sel = O.select_bistride_nodes(_ei(pairs), 5)
    assert sel.tolist() == [1, 3]  # depths from 1: 1,0,1,2,3 -> even: nodes 1, 3 (2/5 = 40 % >= 30 %)
    # star: centre 0 with 9 leaves: even depths = {0} = 10 % < 30 % -> every reachable node
    star = [(0, i) for i in range(1, 10)] + [(i, 0) for i in range(1, 10)]
    assert O.select_bistride_nodes(_ei(star), 10).tolist() == list(range(10))


def test_select_seed_from_pos():
    pos = torch.tensor([[0.0, 0.0], [1.0, 0.0], [2.0, 0.0], [3.0, 0.0], [4.1, 0.0]])
    pairs = [(0, 1), (1, 0), (1, 2), (2, 1), (2, 3), (3, 2), (3, 4), (4, 3)]
    assert O.select_seed(_ei(pairs), 5, pos) == 2  # mean x = 2.02
    assert O.select_bistride_nodes(_ei(pairs), 5, pos).tolist() == [0, 2, 4]


def test_multiscale_graph_structure():
    # triangulated 4x4 grid (odd cycles: even-depth nodes can be adjacent, so coarse edges
    # survive; a bipartite grid would leave none, as the recovered design implies)
    n, pairs = 16, []
    for r in range(4):
        for c in range(4):
            i = 4 * r + c
            if c < 3:
                pairs += [(i, i + 1), (i + 1, i)]
            if r < 3:
                pairs += [(i, i + 4), (i + 4, i)]
            if r < 3 and c < 3:
                pairs += [(i, i + 5), (i + 5, i)]
    ei = _ei(pairs)
    pos = torch.tensor([[c + 0.01 * r, r + 0.003 * c] for r in range(4) for c in range(4)])
    m = O.create_multiscale_graph(ei, pos, n, 2)
    assert len(m["edge_indices"]) == 3 and len(m["node_indices"]) == 2 and len(m["num_nodes"]) == 3
    sel = m["node_indices"][0]
    assert torch.equal(sel, torch.sort(sel).values)
    assert m["num_nodes"][1] == sel.numel()
    e1 = m["edge_indices"][1]
    assert e1.shape[1] > 0 and (e1[0] != e1[1]).all() and int(e1.max()) < m["num_nodes"][1]
    assert torch.equal(m["positions"][1], pos[sel])


def test_unpool_oracle():
    xc = torch.arange(6.0).view(3, 2)
    out = O.unpool(xc, torch.tensor([4, 0, 2]), 5)
    assert out.tolist() == [[2.0, 3.0], [0.0, 0.0], [4.0, 5.0], [0.0, 0.0], [0.0, 1.0]]


def test_modules_construct_and_schema():
    from models.bistride_ops import GMP, Unpool, WeightedEdgeConv
    from models.bsms_mgn import BSMS_MeshGraphNet, BSMSGMP, create_bsms_model_from_config
    w = WeightedEdgeConv(32, 32)
    assert sorted(w.state_dict()) == ["edge_weight_mlp.0.bias", "edge_weight_mlp.0.weight",
                                      "edge_weight_mlp.2.bias", "edge_weight_mlp.2.weight",
                                      "transform.bias", "transform.weight"]
    assert w.edge_weight_mlp[0].weight.shape == (64, 65)
    g = GMP(32, 32, 32)
    assert g.edge_mlp[0].weight.shape == (32, 96) and isinstance(g.edge_mlp[3], torch.nn.LayerNorm)
    b = BSMSGMP(2, 32, 32)
    assert len(b.down_gmps) == 3 and len(b.down_edge_convs) == 2 and len(b.unpools) == 2
    assert isinstance(b.unpools[0], Unpool)
    m = BSMS_MeshGraphNet(6, 4, 4, num_levels=2, latent_dim=32, hidden_dim=32)
    keys = set(m.state_dict())
    assert "bsgmp.bottom_gmp.node_mlp.3.weight" in keys and "decoder.layers.3.bias" in keys
    assert "decoder.layer_norm.weight" not in keys
    m2 = create_bsms_model_from_config({"model": {"input_node_dim": 6, "input_edge_dim": 4, "output_node_dim": 4,
                                                  "num_levels": 2, "latent_dim": 32, "hidden_dim": 32}})
    assert set(m2.state_dict()) == keys
    with pytest.raises(ValueError, match="multi_data must be provided"):
        m(torch.zeros(3, 6), torch.zeros(2, 4), torch.zeros(2, 2, dtype=torch.long))


def test_wec_and_gmp_fail_loudly_on_cpu():
    from models.bistride_ops import GMP, WeightedEdgeConv
    x = torch.zeros(4, 32)
    ei = _ei([(0, 1), (1, 2)])
    with pytest.raises(Exception):
        WeightedEdgeConv(32, 32)(x, ei, torch.zeros(4, 3))
    with pytest.raises(Exception):
        GMP(32, 32, 32)(x, torch.zeros(2, 32), ei)
    with pytest.raises(ValueError, match="Unknown aggregation"):
        WeightedEdgeConv(32, 32, aggr="max")._mean()
