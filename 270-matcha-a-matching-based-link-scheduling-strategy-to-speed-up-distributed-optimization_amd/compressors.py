"""Drop-in compressors (compressors.py:3-19 of the reference) on the GPU."""
import ctypes

import torch

from ._lib import MXError, check, lib, stream_ptr
from .choco import topk_count


# device index -> persistent top-k scratch, zero-filled once (every call leaves it zeroed, so no
# per-call fill of the ~6 P-byte buffer); calls are ordered on the current stream -- concurrent
# get_top_k calls on different streams of one device would share it and are not supported
_WORK = {}
# device index -> host-mapped word the GPU sets when a call's bounded row-barrier wait expired
# (mx_topk_err_forward): (host pointer, device pointer)
_ERR = {}


def _work(device, nbytes):
    w = _WORK.get(device.index)
    if w is None or w.numel() < nbytes:
        w = _WORK[device.index] = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    return w


def _err_word(index):
    e = _ERR.get(index)
    if e is None:
        host, dev = ctypes.POINTER(ctypes.c_int32)(), ctypes.c_void_p()
        check(lib.mx_host_words(1, ctypes.byref(host), ctypes.byref(dev)), "mx_host_words")
        e = _ERR[index] = (host, dev.value)
    return e


def _raise_if_expired(index):
    e = _ERR.get(index)
    if e is not None and e[0][0]:
        row = int(e[0][0]) - 1
        e[0][0] = 0
        _WORK.pop(index, None)    # its histograms may be left half-cleared: the next call starts fresh
        raise MXError(f"get_top_k on cuda:{index}: an earlier call's bounded row-barrier wait expired (row {row}): "
                      "not every block of the row was resident; that call's output was undefined")


def check_top_k(device=None):
    """Synchronise `device` (default: the current one) and raise MXError if a get_top_k call on
    GPU tensors there had a bounded row-barrier wait expire (its output was undefined).  Calls on
    GPU tensors return right after their launch; each one also re-checks the calls before it."""
    d = None if device is None else torch.device(device)
    index = torch.cuda.current_device() if d is None or d.index is None else d.index
    torch.cuda.synchronize(index)
    _raise_if_expired(index)


def get_top_k(x, ratio):
    """Top (1 - ratio) fraction of x by magnitude: k = max(1, int(len * (1 - ratio))).
    Returns (x[indices], indices int64).  Indices come back in ascending order; among equal
    magnitudes at the k-th threshold the lowest indices are kept (the reference's
    torch.topk(sorted=False) / torch.max leave both unspecified).  CPU input (the reference's
    default) is staged to the GPU and the result returned on the input's device (checked before
    returning).  GPU input returns after the launch: an expired bounded wait inside the call is
    raised by the next get_top_k on that device, or by check_top_k()."""
    x_data = x.reshape(-1)
    if x_data.dtype != torch.float32:
        raise TypeError("get_top_k: a float32 tensor is required")
    host = x_data.device.type != "cuda"
    if host:                  # the reference's CPU tensors: staged to the GPU, selected there, returned
        x_data = x_data.to("cuda")
    x_data = x_data.contiguous()
    dev = x_data.device
    _raise_if_expired(dev.index)
    P = x_data.numel()
    k = topk_count(P, ratio)
    vals = torch.empty(k, dtype=torch.float32, device=dev)
    idx = torch.empty(k, dtype=torch.int64, device=dev)
    work = _work(dev, int(lib.mx_topk_work_bytes(P)))
    with torch.cuda.device(dev):   # launch on the stream of the tensor's own device
        check(lib.mx_topk_abs_diff(x_data.data_ptr(), None, P, k, vals.data_ptr(), idx.data_ptr(),
                                   work.data_ptr(), stream_ptr()), "mx_topk_abs_diff")
        if host:
            # the host copy synchronises anyway: also confirm no bounded row-barrier wait expired
            rc = lib.mx_topk_check(work.data_ptr(), 0, 1, P, stream_ptr())
            if rc:
                _WORK.pop(dev.index, None)
                check(rc, "mx_topk_check")
        else:
            check(lib.mx_topk_err_forward(work.data_ptr(), 0, 1, P, _err_word(dev.index)[1], stream_ptr()),
                  "mx_topk_err_forward")
    if host:
        return vals.to(x.device), idx.to(x.device)
    return vals, idx
