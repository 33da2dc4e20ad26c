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


def binary_counter_sum(rows):
    """The binomial tree as mx_mean_rows computes it above 64 rows: a binary counter of partial
    sums, folded right to left at the end (exchange.cpp, mean_to_kernel TREE = 2)."""
    stack, c = {}, 0
    for r in rows:
        p, lvl = r.copy(), 0
        while (c >> lvl) & 1:
            p = stack[lvl] + p
            lvl += 1
        stack[lvl] = p
        c += 1
    acc = None
    for lvl in range(c.bit_length()):
        if (c >> lvl) & 1:
            acc = stack[lvl] if acc is None else stack[lvl] + acc
    return acc
