"""models/mlp.py drop-in (reference: models/mlp.py:5-51).

Module tree and parameter init order are the reference's (so torch.manual_seed gives the
same initial weights); forward runs the whole Linear/ReLU/.../LayerNorm chain as ONE fused
libaerognn kernel (aerognn.functions.MLPFn).
"""
import torch
from torch import nn
import torch.nn.functional as F

from aerognn.core import Pack
from aerognn.functions import ChainSpec, MLPFn


class MLP(nn.Module):
    """Multi-Layer Perceptron with configurable layers and activation."""

    def __init__(self, input_dim: int, hidden_dim: int, output_dim: int, num_hidden_layers: int = 1,
                 activation_fn: str = 'relu', dropout: float = 0.0, use_layer_norm: bool = True):
        super().__init__()
        self.layers = nn.ModuleList()
        self.use_layer_norm = use_layer_norm
        self.layers.append(nn.Linear(input_dim, hidden_dim))                  # mlp.py:22
        for _ in range(num_hidden_layers):
            self.layers.append(nn.Linear(hidden_dim, hidden_dim))             # mlp.py:25-26
        if num_hidden_layers > 0:
            self.layers.append(nn.Linear(hidden_dim, output_dim))             # mlp.py:29-30
        else:
            self.layers[-1] = nn.Linear(input_dim, output_dim)                # mlp.py:31-32 quirk
        if use_layer_norm:
            self.layer_norm = nn.LayerNorm(output_dim)
        self.activation = getattr(F, activation_fn)
        self.dropout = nn.Dropout(dropout)
        self.hidden_dim = hidden_dim
        self.activation_fn = activation_fn
        self._spec = None

    def spec(self):
        if self._spec is None:
            H = self.hidden_dim if len(self.layers) > 1 else max(32, ((self.layers[0].weight.shape[0] + 31) // 32) * 32)
            if H not in (32, 64, 128):
                raise NotImplementedError(f"aerognn fused MLP supports hidden_dim 32/64/128, got {H}")
            lins = [(m.weight, m.bias) for m in self.layers]
            ln = (self.layer_norm.weight, self.layer_norm.bias) if self.use_layer_norm else None
            self._spec = ChainSpec(lins, ln, H, Pack(), act=self.activation_fn)
            self._spec.check_hidden()
        return self._spec

    def forward(self, x):
        if x.dtype == torch.float64:  # train.py precision "double": agn_f64_* kernels (aerognn/f64.py)
            from aerognn import f64
            return f64.mlp_forward(self, x)
        if self.training and self.dropout.p > 0:
            raise NotImplementedError("aerognn fused MLP: dropout > 0 in training is not implemented")
        s = self.spec()
        s.pack.update(x.dtype, x.device)
        return MLPFn.apply(x, s, torch.is_grad_enabled(), None, *s.params())

    def forward_rows(self, x, rows):
        """self.forward(x[rows]) with the row gather fused into the first layer's input loads (the
        kernel reads row rows[i] for output row i; no gathered copy): the edge encoder on the
        caller's edge features in a level's receiver-grouped order."""
        if x.dtype == torch.float64:
            from aerognn import f64
            return f64.mlp_forward(self, x, rows)
        if self.training and self.dropout.p > 0:
            raise NotImplementedError("aerognn fused MLP: dropout > 0 in training is not implemented")
        s = self.spec()
        s.pack.update(x.dtype, x.device)
        return MLPFn.apply(x, s, torch.is_grad_enabled(), rows, *s.params())
