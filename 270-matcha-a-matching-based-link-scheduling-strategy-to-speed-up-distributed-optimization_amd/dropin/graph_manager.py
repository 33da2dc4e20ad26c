"""Drop-in for the reference's graph_manager.py (see the package's graph_manager module)."""
from _mx_pkg import PKG

GraphProcessor = PKG.GraphProcessor
FixedProcessor = PKG.FixedProcessor
MatchaProcessor = PKG.MatchaProcessor
