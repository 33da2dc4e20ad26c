"""CPU: the summation orders of the centralized communicator's reference-order all-reduce.

mx_mean_rows runs mpi4py's binomial-tree order (communicator.py:61, comm.allreduce under
rc.fast_reduce) over a register array up to 64 rows and as a binary counter of partial sums above
(exchange.cpp mean_to_kernel TREE = 2).  The two statements must be the same order: checked
here bit for bit on fp32 rows of mixed magnitudes for every row count 1..300.  (The mpi4py order
itself is restated from its published algorithm -- mpi4py is not installed: parity unpinned
against mpi4py.)"""
import numpy as np

from reforder import binary_counter_sum, mpi4py_sum


def test_binary_counter_equals_binomial_tree():
    rng = np.random.RandomState(7)
    for n in range(1, 301):
        rows = [(rng.standard_normal(97) * 10.0 ** rng.randint(-3, 4)).astype(np.float32) for _ in range(n)]
        a = mpi4py_sum(rows, "tree")
        b = binary_counter_sum(rows)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), n
