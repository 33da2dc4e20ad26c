"""Python restatement of the round-plan contract (plan.hip / mx_plan_build) -- test helper.

For iteration flags `flags_row`, rows [row_base, row_base + n_local) of `partner` [M][n]:
each local row's partners in ascending matching order as slots (slot < n_local: local row,
slot >= n_local: receive-slab row of a distinct remote worker, numbered by first appearance in
(matching asc, sender id asc) order), and the
selfweight f32(1 - degree * alpha) (communicator.py:99-117)."""
import numpy as np


def py_plan(flags_row, partner, row_base, n_local, alpha):
    M, n = partner.shape
    src = [[] for _ in range(n_local)]
    senders = []                      # slab slot -> worker id
    for g in range(M):
        if not flags_row[g]:
            continue
        for p in range(n):
            q = int(partner[g, p])
            if not (row_base <= q < row_base + n_local):
                continue
            if row_base <= p < row_base + n_local:
                src[q - row_base].append(p - row_base)
            else:                     # one slab slot per distinct remote worker
                if p not in senders:
                    senders.append(p)
                src[q - row_base].append(n_local + senders.index(p))
    sw = [np.float32(1.0 - len(s) * alpha) for s in src]
    return int(any(flags_row)), len(senders), src, sw, senders
