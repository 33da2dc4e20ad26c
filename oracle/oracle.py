"""ctypes front end for the CPU oracle (liboracle.so, built from matcha_oracle.c).

TEST INFRASTRUCTURE ONLY -- the parity checker.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.  The product package never imports it.

Each function restates a reference function; the file:line it follows is in
matcha_oracle.c's header and in the docstrings below.  Pinned against the golden fixtures
emitted by running the reference itself (tests/golden/make_golden.py); see
tests/test_oracle.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(HERE, "liboracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.orc_matcha_flags.argtypes = [_u32p, ctypes.POINTER(ctypes.c_int), _f64p, ctypes.c_int,
                                       ctypes.c_int64, _u8p]
        L.orc_fixed_flags.argtypes = [_u32p, ctypes.POINTER(ctypes.c_int), ctypes.c_double,
                                      ctypes.c_int64, _u8p]
        L.orc_mt_seed_key.argtypes = [ctypes.c_uint32, _u32p, ctypes.POINTER(ctypes.c_int)]
        L.orc_decen_round.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int64, _i32p, _u8p,
                                      ctypes.c_int, ctypes.c_double]
        L.orc_topk_abs.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int64, _f32p, _i64p]
        L.orc_topk_abs.restype = ctypes.c_int
        L.orc_topk_abs_sort.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int64, _f32p, _i64p]
        L.orc_topk_abs_sort.restype = ctypes.c_int
        L.orc_choco_round.argtypes = [_f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int64, _i32p,
                                      _u8p, ctypes.c_int, ctypes.c_double, ctypes.c_int64,
                                      ctypes.c_double]
        L.orc_choco_round.restype = ctypes.c_int
        L.orc_choco_averaging.argtypes = L.orc_choco_round.argtypes
        L.orc_choco_averaging.restype = ctypes.c_int
        L.orc_baseline_rounds.argtypes = [ctypes.POINTER(ctypes.c_void_p), _i64p, ctypes.c_int,
                                          ctypes.c_int, _i32p, _u8p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_double, _f32p, ctypes.c_int]
        L.orc_baseline_rounds.restype = ctypes.c_int
        L.orc_central_mean.argtypes = [_f32p, ctypes.c_int, ctypes.c_int64, ctypes.c_int, _f32p]
        L.orc_central_mean.restype = ctypes.c_int
        L.orc_synth.argtypes = [ctypes.c_uint64, ctypes.c_int64, _f32p]
        L.orc_num_threads.restype = ctypes.c_int
        _lib = L
    return _lib


# ---------------------------------------------------------------------------- schedule
def mt_seed(seed):
    """np.random.seed(seed) -> (key uint32[624], pos)."""
    key = np.zeros(624, np.uint32)
    pos = ctypes.c_int(0)
    lib().orc_mt_seed_key(seed, key, ctypes.byref(pos))
    return key, pos.value


def matcha_flags(key, pos, p, T):
    """MatchaProcessor.set_flags(T) (graph_manager.py:298-309) from MT state (key, pos).
    Returns (flags uint8 [T][M], key', pos')."""
    key = np.array(key, dtype=np.uint32, copy=True)
    p = np.ascontiguousarray(p, dtype=np.float64)
    M = p.shape[0]
    out = np.zeros((T, M), np.uint8)
    c = ctypes.c_int(pos)
    lib().orc_matcha_flags(key, ctypes.byref(c), p, M, T, out)
    return out, key, c.value


def fixed_flags(key, pos, budget, T):
    """FixedProcessor.set_flags(T) (graph_manager.py:208-225)."""
    key = np.array(key, dtype=np.uint32, copy=True)
    out = np.zeros((T, 2), np.uint8)
    c = ctypes.c_int(pos)
    lib().orc_fixed_flags(key, ctypes.byref(c), float(budget), T, out)
    return out, key, c.value


# ---------------------------------------------------------------------------- gossip
def decen_round(X, partner, flags, alpha):
    """decenCommunicator round for all workers (communicator.py:87-158). X: [n][P] f32."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, P = X.shape
    partner = np.ascontiguousarray(partner, dtype=np.int32)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    Y = np.empty_like(X)
    lib().orc_decen_round(X, Y, n, P, partner, flags, partner.shape[0], float(alpha))
    return Y


def topk_k(P, ratio):
    """compressors.py:11 -- k = max(1, int(len * (1 - ratio)))."""
    return max(1, int(P * (1 - ratio)))


def topk_abs(x, k, sort=False):
    """compressors.get_top_k (compressors.py:3-19), index-sorted; ties -> lowest index.
    sort=True: the full-sort statement of the same rule (cross-check; slow at large P)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    vals = np.empty(k, np.float32)
    idx = np.empty(k, np.int64)
    f = lib().orc_topk_abs_sort if sort else lib().orc_topk_abs
    rc = f(x, x.shape[0], k, vals, idx)
    assert rc == 0, rc
    return vals, idx


def choco_round(X, XH, S, partner, flags, alpha, k, gamma, skip_empty=True):
    """ChocoCommunicator round for all workers (communicator.py:175-268); state in place.
    skip_empty=False: prepare_comm_buffer + averaging(flags) called directly -- a row with no
    active matching still applies every worker's own message (communicator.py:175-230)."""
    n, P = X.shape
    for a in (X, XH, S):
        assert a.dtype == np.float32 and a.flags.c_contiguous
    partner = np.ascontiguousarray(partner, dtype=np.int32)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    f = lib().orc_choco_round if skip_empty else lib().orc_choco_averaging
    rc = f(X, XH, S, n, P, partner, flags, partner.shape[0], float(alpha), int(k), float(gamma))
    assert rc == 0, rc


def central_mean(X, order="tree"):
    """centralizedCommunicator round (communicator.py:46-76): every worker's vector becomes the
    fp32 sum of all workers' vectors in mpi4py's object-allreduce order ("tree": binomial tree,
    its default; "sequential": rank order), divided by n.  X: [n][P] f32 -> the mean [P]."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    n, P = X.shape
    out = np.empty(P, np.float32)
    rc = lib().orc_central_mean(X, n, P, {"tree": 0, "sequential": 1}[order], out)
    assert rc == 0, rc
    return out


def baseline_rounds(segs, partner, flags, alpha, threads=0):
    """Timed CPU port of the reference per-rank sequence.  segs: list over workers of lists of
    float32 arrays (the model tensors).  flags: [rounds][M].  Mutates segs in place."""
    n = len(segs)
    nseg = len(segs[0])
    seg_len = np.array([a.size for a in segs[0]], np.int64)
    P = int(seg_len.sum())
    ptrs = (ctypes.c_void_p * (n * nseg))()
    for i in range(n):
        for s in range(nseg):
            a = segs[i][s]
            assert a.dtype == np.float32 and a.flags.c_contiguous
            ptrs[i * nseg + s] = a.ctypes.data
    scratch = np.empty(n * 3 * P, np.float32)
    partner = np.ascontiguousarray(partner, dtype=np.int32)
    flags = np.ascontiguousarray(flags, dtype=np.uint8).reshape(-1, partner.shape[0])
    rc = lib().orc_baseline_rounds(ptrs, seg_len, nseg, n, partner, flags, partner.shape[0],
                                   flags.shape[0], float(alpha), scratch, int(threads))
    assert rc == 0


def num_threads():
    return lib().orc_num_threads()


# ---------------------------------------------------------------------------- inputs
def synth(seed, n):
    """splitmix64 counter -> fp32 uniform[-1,1) (SURVEY.md §8d synthetic inputs)."""
    out = np.empty(n, np.float32)
    lib().orc_synth(seed, n, out)
    return out


def synth_np(seed, n):
    """Same generator in numpy (cross-check of orc_synth)."""
    return synth_at(seed, np.arange(n, dtype=np.int64))


def synth_at(seed, cols):
    """synth(seed, n)[cols] without generating the whole row (the generator is counter-based)."""
    i = np.asarray(cols, dtype=np.uint64) + np.uint64(1)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    m = (z >> np.uint64(40)).astype(np.float32)
    return (m * np.float32(2.0 ** -23) - np.float32(1.0)).astype(np.float32)
