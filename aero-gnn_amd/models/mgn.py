"""models/mgn.py drop-in (reference: models/mgn.py:9-139): encoders -> processor_size x
MeshGraphNetLayer -> decoder. The edge latents are kept receiver-grouped (CSC) for the whole
processor; the graph is grouped once per forward (one radix sort)."""
import torch
from torch import nn

from aerognn.graph import Level
from models.mlp import MLP
from models.mgnLayer import MeshGraphNetLayer


class MeshGraphNet(nn.Module):
    """Complete MeshGraphNet model for mesh-based physical simulations."""

    def __init__(self, input_node_dim: int, input_edge_dim: int, output_node_dim: int, processor_size: int = 15,
                 activation_fn: str = 'relu', num_hidden_layers_node_processor: int = 1,
                 num_hidden_layers_edge_processor: int = 1, hidden_dim_processor: int = 128,
                 num_hidden_layers_node_encoder: int = 1, hidden_dim_node_encoder: int = 128,
                 num_hidden_layers_edge_encoder: int = 1, hidden_dim_edge_encoder: int = 128,
                 aggregation: str = 'sum', hidden_dim_decoder: int = 128, num_hidden_layers_decoder: int = 1,
                 dropout: float = 0.0, do_concat_trick: bool = False):
        super().__init__()
        self.node_encoder = MLP(input_node_dim, hidden_dim=hidden_dim_node_encoder, output_dim=hidden_dim_processor,
                                num_hidden_layers=num_hidden_layers_node_encoder, activation_fn=activation_fn,
                                dropout=dropout, use_layer_norm=True)
        self.edge_encoder = MLP(input_edge_dim, hidden_dim=hidden_dim_edge_encoder, output_dim=hidden_dim_processor,
                                num_hidden_layers=num_hidden_layers_edge_encoder, activation_fn=activation_fn,
                                dropout=dropout, use_layer_norm=True)
        self.layers = nn.ModuleList([
            MeshGraphNetLayer(node_dim=hidden_dim_processor, edge_dim=hidden_dim_processor,
                              hidden_dim=hidden_dim_processor,
                              num_hidden_layers_node_processor=num_hidden_layers_node_processor,
                              num_hidden_layers_edge_processor=num_hidden_layers_edge_processor,
                              activation_fn=activation_fn, use_layer_norm=True, aggregation=aggregation,
                              do_concat_trick=do_concat_trick)
            for _ in range(processor_size)])
        self.decoder = MLP(input_dim=hidden_dim_processor, hidden_dim=hidden_dim_decoder, output_dim=output_node_dim,
                           num_hidden_layers=num_hidden_layers_decoder, activation_fn=activation_fn,
                           use_layer_norm=False)

    def forward(self, node_attr: torch.Tensor, edge_attr: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        level = Level.from_edge_index(edge_index, node_attr.shape[0])
        node_hidden = self.node_encoder(node_attr)
        edge_hidden = self.edge_encoder.forward_rows(edge_attr, level.perm)
        for layer in self.layers:
            node_hidden, edge_hidden = layer.forward_level(node_hidden, edge_hidden, level)
        return self.decoder(node_hidden)
