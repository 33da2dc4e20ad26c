"""Locates the package for the drop-in shims.  Put this directory on sys.path (PYTHONPATH) in
place of the reference's directory and `from graph_manager import ...` /
`from communicator import ...` in train_mpi.py resolve to the MI355X implementation."""
import importlib
import os
import sys

PKG_NAME = "270-matcha-a-matching-based-link-scheduling-strategy-to-speed-up-distributed-optimization_amd"
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
PKG = importlib.import_module(PKG_NAME)
