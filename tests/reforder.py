"""Summation orders of the reference's object all-reduce (test helper, numpy only)."""


def mpi4py_sum(rows, order):
    """The reference's comm.allreduce(x, op=MPI.SUM) (communicator.py:61) summation order, fp32:
    "tree" = mpi4py's default binomial reduction to rank 0, "sequential" = rank-order fold."""
    v = [r.copy() for r in rows]
    if order == "sequential":
        acc = v[0]
        for r in v[1:]:
            acc = acc + r
        return acc
    m = 1
    while m < len(v):
        for r in range(0, len(v), 2 * m):
            if r + m < len(v):
                v[r] = v[r] + v[r + m]
        m *= 2
    return v[0]
