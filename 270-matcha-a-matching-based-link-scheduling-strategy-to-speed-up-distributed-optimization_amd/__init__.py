"""MI355X-native MATCHA / D-PSGD / ChocoSGD gossip hot path (gfx950 HIP kernels + RCCL).

Drop-in surface of the reference (graph_manager.py, communicator.py, comm_helpers.py,
compressors.py) plus the multi-worker groups the MI355X layout is built around.  The native
library (_native/libmatcha_gossip.so, include/matcha_gossip.h) is required: importing this
package without it fails.
"""
from ._lib import MXError, lib
from .graph_manager import GraphProcessor, FixedProcessor, MatchaProcessor
from .engine import GossipEngine, VirtualWorkerGroup, RcclComm, PullTransport, Layout, partition, pull_stats
from .choco import ChocoWorkerGroup, topk_count
from .communicator import Communicator, decenCommunicator, ChocoCommunicator, centralizedCommunicator
from .comm_helpers import flatten_tensors, unflatten_tensors, scatter_tensors
from .compressors import get_top_k, check_top_k
from .topologies import select_graph, erdos_renyi, GRAPH_SIZES
from . import solver
from . import harness
from . import placement
from .placement import best_placement, placement_cost

__all__ = [
    "MXError", "lib", "GraphProcessor", "FixedProcessor", "MatchaProcessor", "GossipEngine",
    "VirtualWorkerGroup", "RcclComm", "PullTransport", "Layout", "partition", "pull_stats", "ChocoWorkerGroup", "topk_count",
    "Communicator", "decenCommunicator", "ChocoCommunicator", "centralizedCommunicator",
    "flatten_tensors", "unflatten_tensors", "scatter_tensors", "get_top_k", "check_top_k", "select_graph",
    "erdos_renyi", "GRAPH_SIZES", "solver", "harness", "placement", "best_placement", "placement_cost",
]
