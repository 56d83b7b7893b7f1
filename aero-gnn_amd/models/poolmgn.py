"""models/poolmgn.py drop-in (reference: models/poolmgn.py:11-158): MeshGraphNet with a global
pooled context. A global encoder MLP (no LayerNorm) runs on the raw node features, is pooled per
graph (torch_geometric global_{mean,max,add}_pool), broadcast back to the nodes and concatenated
to the node features before the node encoder; then processor_size MeshGraphNetLayers and the
decoder, as in models/mgn.py.

Constructor, module registration order (state_dict keys) and forward signature are the
reference's. The pooling runs on libaerognn segment kernels (GlobalPoolFn: fixed member order
sum / mean, first-argmax max), the broadcast is a row gather whose backward is a per-graph
segment sum (BroadcastRowsFn), and the processor shares one receiver-grouped Level across its
layers (the reference rebuilds nothing either: its per-layer cost is the scatter).
"""
import torch
from torch import nn

from aerognn.core import require_device
from aerognn.functions import BroadcastRowsFn, GlobalPoolFn, GraphGroups
from aerognn.graph import Level
from models.mlp import MLP
from models.mgnLayer import MeshGraphNetLayer


class poolMGN(nn.Module):
    """Complete MeshGraphNet model for mesh-based physical simulations."""

    def __init__(self, input_node_dim: int, input_edge_dim: int, output_node_dim: int, processor_size: int = 15,
                 activation_fn: str = 'relu', num_hidden_layers_node_processor: int = 1,
                 num_hidden_layers_edge_processor: int = 1, hidden_dim_processor: int = 128,
                 num_hidden_layers_node_encoder: int = 1, hidden_dim_node_encoder: int = 128,
                 num_hidden_layers_edge_encoder: int = 1, hidden_dim_edge_encoder: int = 128,
                 aggregation: str = 'sum', hidden_dim_decoder: int = 128, num_hidden_layers_decoder: int = 1,
                 global_pool_method: str = 'mean', num_hidden_layers_global_encoder: int = 1, global_dim: int = 128,
                 dropout: float = 0.0):
        super().__init__()
        if global_pool_method not in ('mean', 'max', 'add'):
            raise ValueError(f"Unsupported global pooling method: {global_pool_method}")  # poolmgn.py:38-45
        self.global_pool_method = global_pool_method
        self.node_encoder = MLP(input_node_dim + global_dim, hidden_dim=hidden_dim_node_encoder,
                                output_dim=hidden_dim_processor, num_hidden_layers=num_hidden_layers_node_encoder,
                                activation_fn=activation_fn, dropout=dropout, use_layer_norm=True)
        self.edge_encoder = MLP(input_edge_dim, hidden_dim=hidden_dim_edge_encoder, output_dim=hidden_dim_processor,
                                num_hidden_layers=num_hidden_layers_edge_encoder, activation_fn=activation_fn,
                                dropout=dropout, use_layer_norm=True)
        self.global_encoder = MLP(input_node_dim, hidden_dim=global_dim, output_dim=global_dim,
                                  num_hidden_layers=num_hidden_layers_global_encoder, activation_fn=activation_fn,
                                  dropout=dropout, use_layer_norm=False)
        self.layers = nn.ModuleList([
            MeshGraphNetLayer(node_dim=hidden_dim_processor, edge_dim=hidden_dim_processor,
                              hidden_dim=hidden_dim_processor,
                              num_hidden_layers_node_processor=num_hidden_layers_node_processor,
                              num_hidden_layers_edge_processor=num_hidden_layers_edge_processor,
                              activation_fn=activation_fn, use_layer_norm=True, aggregation=aggregation)
            for _ in range(processor_size)])
        self.decoder = MLP(input_dim=hidden_dim_processor, hidden_dim=hidden_dim_decoder, output_dim=output_node_dim,
                           num_hidden_layers=num_hidden_layers_decoder, activation_fn=activation_fn,
                           use_layer_norm=False)

    def forward(self, node_attr: torch.Tensor, edge_attr: torch.Tensor, edge_index: torch.Tensor,
                batch: torch.Tensor = None):
        require_device(node_attr, edge_attr, edge_index, batch)
        n = node_attr.size(0)
        groups = GraphGroups(batch, n, node_attr.device)
        g = self.global_encoder(node_attr)
        g = GlobalPoolFn.apply(g, groups, self.global_pool_method)   # [G, global_dim]
        g = BroadcastRowsFn.apply(g, groups)                          # [N, global_dim]
        x = self.node_encoder(torch.cat((node_attr, g), dim=-1))
        level = Level.from_edge_index(edge_index, n)
        e = self.edge_encoder.forward_rows(edge_attr, level.perm)
        for layer in self.layers:
            x, e = layer.forward_level(x, e, level)
        return self.decoder(x)
