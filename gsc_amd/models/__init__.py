"""GNN embedder (GATv2), actor and critic."""
from .gnn import GATv2Params, GNNEmbedder, gatv2_dense_reference
from .graphs import GraphSet
from .nets import Actor, MaskedInputMLP, QNetwork, count_params
