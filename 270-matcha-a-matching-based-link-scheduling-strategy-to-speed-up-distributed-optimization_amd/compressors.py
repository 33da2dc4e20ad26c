"""Drop-in compressors (compressors.py:3-19 of the reference) on the GPU."""
import torch

from ._lib import check, lib, stream_ptr
from .choco import topk_count


# device index -> persistent top-k scratch, zero-filled once (every call leaves it zeroed, so no
# per-call fill of the ~6 P-byte buffer); calls are ordered on the current stream -- concurrent
# get_top_k calls on different streams of one device would share it and are not supported
_WORK = {}


def _work(device, nbytes):
    w = _WORK.get(device.index)
    if w is None or w.numel() < nbytes:
        w = _WORK[device.index] = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    return w


def get_top_k(x, ratio):
    """Top (1 - ratio) fraction of x by magnitude: k = max(1, int(len * (1 - ratio))).
    Returns (x[indices], indices int64).  Indices come back in ascending order; among equal
    magnitudes at the k-th threshold the lowest indices are kept (the reference's
    torch.topk(sorted=False) / torch.max leave both unspecified).  CPU input (the reference's
    default) is staged to the GPU and the result returned on the input's device."""
    x_data = x.reshape(-1)
    if x_data.dtype != torch.float32:
        raise TypeError("get_top_k: a float32 tensor is required")
    host = x_data.device.type != "cuda"
    if host:                  # the reference's CPU tensors: staged to the GPU, selected there, returned
        x_data = x_data.to("cuda")
    x_data = x_data.contiguous()
    P = x_data.numel()
    k = topk_count(P, ratio)
    vals = torch.empty(k, dtype=torch.float32, device=x_data.device)
    idx = torch.empty(k, dtype=torch.int64, device=x_data.device)
    work = _work(x_data.device, int(lib.mx_topk_work_bytes(P)))
    with torch.cuda.device(x_data.device):   # launch on the stream of the tensor's own device
        check(lib.mx_topk_abs_diff(x_data.data_ptr(), None, P, k, vals.data_ptr(), idx.data_ptr(),
                                   work.data_ptr(), stream_ptr()), "mx_topk_abs_diff")
    if host:
        # the host copy synchronises anyway: also confirm no bounded row-barrier wait expired
        check(lib.mx_topk_check(work.data_ptr(), 0, 1, P, stream_ptr()), "mx_topk_check")
        return vals.to(x.device), idx.to(x.device)
    return vals, idx
