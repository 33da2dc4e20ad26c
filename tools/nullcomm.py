"""A transport that skips the transfer: a rank's share of an N-GPU layout timed on one GPU
(received rows / messages hold whatever valid stand-ins the caller put there)."""


class NullComm:
    def __init__(self, rank, nranks):
        self.rank, self.nranks, self.handle = rank, nranks, None

    def exchange_round(self, engine, it, row_ptrs, slab_ptr, slab_ld_bytes, row_bytes):
        """Reports the receive count the native exchange plan would post."""
        return int(sum(1 for op in engine.exchange_plan(it) if op[0] == 1))
