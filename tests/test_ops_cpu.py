"""torch.ops.aerognn.* registration (aerognn/ops.py): schemas, fake kernels for
shape propagation (FakeTensorMode / torch.compile tracing) and the no-CPU-fallback rule. The
numerics run on the GPU (tests/test_gpu_ops.py)."""
import pytest
import torch

OPS = ("scatter_sum", "gather_rows", "scatter_max", "scatter_max_backward", "edge_features", "group_ptr")


def test_ops_registered_with_schema():
    import aerognn.ops  # noqa: F401  (registers the operators)
    for name in OPS:
        op = getattr(torch.ops.aerognn, name)
        assert str(op.default._schema).startswith(f"aerognn::{name}(")


def test_fake_kernels_propagate_shapes():
    import aerognn.ops  # noqa: F401
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        x = torch.empty(10, 4, dtype=torch.bfloat16)
        i = torch.zeros(10, dtype=torch.long)
        assert torch.ops.aerognn.scatter_sum(x, i, 3, True).shape == (3, 4)
        assert torch.ops.aerognn.gather_rows(x, i).shape == (10, 4)
        out, arg = torch.ops.aerognn.scatter_max(x, i, 5)
        assert out.shape == (5, 4) and out.dtype == torch.bfloat16 and arg.dtype == torch.int64
        assert torch.ops.aerognn.edge_features(torch.empty(5, 3), torch.zeros(2, 7, dtype=torch.long)).shape == (7, 4)


def test_autograd_formulas_registered():
    import aerognn.ops  # noqa: F401
    for name in ("scatter_sum", "gather_rows", "scatter_max"):
        assert torch._C._dispatch_has_kernel_for_dispatch_key(f"aerognn::{name}", "Autograd"), name


@pytest.mark.parametrize("name", ["scatter_sum", "gather_rows", "scatter_max"])
def test_cpu_tensors_raise(name):
    import aerognn.ops  # noqa: F401
    x, i = torch.ones(3, 2), torch.zeros(3, dtype=torch.long)
    args = {"scatter_sum": (x, i, 1, False), "gather_rows": (x, i), "scatter_max": (x, i, 1)}[name]
    with pytest.raises(RuntimeError, match="MI355X"):
        getattr(torch.ops.aerognn, name)(*args)
