"""MI355X-native GNN message passing for the elliptic-gnn-project hot path.

Drop-in for ``torch_geometric.nn.{SAGEConv, GCNConv, GATConv}`` as used by the reference's
``src/models/gnn.py``: hand-written gfx950 HIP kernels (libgnnmp.so, C ABI in
include/gnnmp.h) behind PyG-compatible modules.  Importing the package does not touch the
GPU; the library is loaded on first use and there is no CPU fallback.
"""
from .conv import GATConv, GCNConv, SAGEConv  # noqa: F401
from .gnn import GATNet, GCNNet, SAGENet, SAGEResBNNet  # noqa: F401

__version__ = "0.1.0"
