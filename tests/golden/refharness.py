"""Harness that imports the READ-ONLY reference (/root/reference) in this container only.

Test infrastructure, used solely by ``make_golden.py`` to emit the committed fixtures
under ``tests/golden/``.  Nothing in the product, in ``-m gpu`` tests, in ``smoke()`` or in
``bench.py`` imports this file; the reference does not exist on the GPU box.

What it provides (SURVEY.md §4 "What this container can do instead"):
  * in-process stub modules for the absent ``mpi4py`` / ``cvxpy`` / ``torchvision``
    (they fail with an ordinary ModuleNotFoundError otherwise);
  * a networkx>=3 shim for ``nx.laplacian_matrix(G, nodelist)``, which raises when a node of
    ``nodelist`` is missing from ``G`` (graph_manager.py:91); networkx 2.x gave zero rows;
  * ``FakeWorld``: a threaded in-process stand-in for ``MPI.COMM_WORLD`` (one thread per rank,
    a ``threading.Barrier``, one queue per (src, dst) pair, pickle round trip on ``sendrecv``
    exactly as mpi4py's lowercase API does).
"""
import os
import pickle
import queue
import sys
import threading
import types

REF = "/root/reference"


class FakeWorld:
    """Thread-per-rank stand-in for ``MPI.COMM_WORLD`` (communicator.py:14)."""

    def __init__(self, size):
        self.size = size
        self._barrier = threading.Barrier(size)
        self._q = {(s, d): queue.Queue() for s in range(size) for d in range(size)}
        self._tls = threading.local()
        self._slots = [None] * size

    # rank of the calling thread
    def Get_rank(self):
        return self._tls.rank

    def Get_size(self):
        return self.size

    def bind(self, rank):
        self._tls.rank = rank

    def barrier(self):
        self._barrier.wait()

    def sendrecv(self, sendobj, dest, sendtag=0, recvbuf=None, source=None, recvtag=None, status=None):
        me = self._tls.rank
        self._q[(me, dest)].put(pickle.dumps(sendobj))
        return pickle.loads(self._q[(source, me)].get())

    def allreduce(self, sendobj, op=None):
        me = self._tls.rank
        self._slots[me] = pickle.loads(pickle.dumps(sendobj))
        self._barrier.wait()
        acc = None
        for r in range(self.size):          # rank order
            acc = self._slots[r].clone() if acc is None else acc + self._slots[r]
        self._barrier.wait()
        return acc


_WORLD = None


def install(size):
    """Install stubs + shims and import the reference modules. Returns a namespace."""
    global _WORLD
    sys.dont_write_bytecode = True          # never write __pycache__ into /root/reference
    _WORLD = FakeWorld(size)

    mpi4py = types.ModuleType("mpi4py")
    MPI = types.ModuleType("mpi4py.MPI")
    MPI.COMM_WORLD = _WORLD
    MPI.SUM = "SUM"
    mpi4py.MPI = MPI
    sys.modules["mpi4py"] = mpi4py
    sys.modules["mpi4py.MPI"] = MPI
    sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
    tv = types.ModuleType("torchvision")
    tv.datasets = types.ModuleType("torchvision.datasets")
    tv.transforms = types.ModuleType("torchvision.transforms")
    tv.models = types.ModuleType("torchvision.models")
    for m in (tv, tv.datasets, tv.transforms, tv.models):
        sys.modules.setdefault(m.__name__, m)

    import networkx as nx
    if not getattr(nx.laplacian_matrix, "_graft_shim", False):
        _orig = nx.laplacian_matrix

        def laplacian_matrix(G, nodelist=None, *a, **kw):
            if nodelist is not None:
                G = G.copy()
                G.add_nodes_from(nodelist)
            return _orig(G, nodelist, *a, **kw)

        laplacian_matrix._graft_shim = True
        nx.laplacian_matrix = laplacian_matrix

    if REF not in sys.path:
        sys.path.insert(0, REF)
    import comm_helpers, compressors, graph_manager, communicator  # noqa: E401
    try:
        import util  # noqa: F401
    except Exception:  # util pulls in models/torchvision at import; select_graph is all we need
        util = None
    for mod in (graph_manager, communicator):
        mod.MPI.COMM_WORLD = _WORLD
    ns = types.SimpleNamespace(comm_helpers=comm_helpers, compressors=compressors,
                               graph_manager=graph_manager, communicator=communicator,
                               util=util, world=_WORLD)
    return ns


def new_world(size):
    """Replace ``MPI.COMM_WORLD`` with a fresh FakeWorld of ``size`` ranks (before constructing
    communicators: they capture it at __init__, communicator.py:14)."""
    global _WORLD
    _WORLD = FakeWorld(size)
    sys.modules["mpi4py.MPI"].COMM_WORLD = _WORLD
    return _WORLD


def run_ranks(size, fn):
    """Run ``fn(rank)`` on ``size`` threads bound to FakeWorld ranks; return results by rank."""
    out = [None] * size
    err = []

    def body(r):
        _WORLD.bind(r)
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            err.append((r, e))
            _WORLD._barrier.abort()

    ths = [threading.Thread(target=body, args=(r,)) for r in range(size)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if err:
        raise err[0][1]
    return out
