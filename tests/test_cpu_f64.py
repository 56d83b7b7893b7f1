"""float64 mode plumbing on the CPU (no kernel launches): dtype code, chain binding of the
reference modules (mlp.py:21-35, mgnLayer.py:72-90), and no CPU fallback."""
import pytest
import torch


def test_f64_dtype_code():
    from aerognn import _lib as L
    from aerognn.core import dt_code
    assert dt_code(torch.float64) == L.F64 == 3


def test_f64_chain_binding_follows_reference_modules():
    from aerognn import f64
    from models.mgnLayer import MeshGraphNetLayer
    from models.mlp import MLP
    torch.manual_seed(0)
    m = MLP(10, 32, 8, num_hidden_layers=2).double()
    ch = f64.mlp_chain(m)
    assert [w for w, _ in ch.lins] == [l.weight for l in m.layers]
    assert ch.params() == [p for l in m.layers for p in (l.weight, l.bias)] + [m.layer_norm.weight, m.layer_norm.bias]
    layer = MeshGraphNetLayer(32, 32, 32, 1, 1, do_concat_trick=True).double()
    eb = layer.edge_block
    ec = f64.edge_chain(eb)
    assert ec.lins[0][0] is eb.edge_lin and ec.lins[0][1] is None
    assert len(ec.lins) == 3 and ec.ln is not None  # W_e, one hidden Linear, the output Linear; LN


def test_f64_has_no_cpu_fallback():
    from models.mlp import MLP
    m = MLP(4, 32, 4, num_hidden_layers=1).double()
    with pytest.raises(Exception):
        m(torch.randn(5, 4, dtype=torch.float64))  # CPU tensors: the library path refuses them
