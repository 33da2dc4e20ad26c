"""Drop-in comm_helpers (comm_helpers.py:12-75 of the reference).

flatten_tensors concatenates device tensors with one multi-tensor gather launch (mx_gather) in
place of torch.cat; unflatten_tensors returns narrow().view_as() views exactly as the reference
does (no data movement, any device).
"""
import numpy as np
import torch

from ._lib import check, lib, stream_ptr


def _offsets(tensors):
    off = np.zeros(len(tensors) + 1, dtype=np.int64)
    for i, t in enumerate(tensors):
        off[i + 1] = off[i] + t.numel()
    return off


def flatten_tensors(tensors):
    """comm_helpers.py:12-30: one contiguous 1-D float32 buffer holding the tensors in order.
    A single tensor is copied too (the reference returns view(-1).clone())."""
    tensors = list(tensors)
    if not tensors:
        raise ValueError("flatten_tensors needs at least one tensor")
    dev = tensors[0].device
    for t in tensors:
        if t.dtype != torch.float32 or t.device != dev:
            raise TypeError("flatten_tensors: float32 tensors on one device required")
    if dev.type != "cuda":    # the reference's CPU tensors: gathered on the GPU, returned on the CPU
        return flatten_tensors([t.to("cuda") for t in tensors]).to(dev)
    src = [t.contiguous() for t in tensors]
    off = _offsets(src)
    total = int(off[-1])
    flat = torch.empty(total, dtype=torch.float32, device=src[0].device)
    if total:
        ptrs = torch.tensor([t.data_ptr() for t in src], dtype=torch.int64, device=flat.device)
        offd = torch.from_numpy(off).to(flat.device)
        with torch.cuda.device(flat.device):     # the stream of the tensors' own device
            check(lib.mx_gather(ptrs.data_ptr(), offd.data_ptr(), len(src), total, flat.data_ptr(),
                                stream_ptr()), "mx_gather")
    return flat


def unflatten_tensors(flat, tensors):
    """comm_helpers.py:33-56: views of `flat` shaped like `tensors`."""
    outputs = []
    offset = 0
    for tensor in tensors:
        numel = tensor.numel()
        outputs.append(flat.narrow(0, offset, numel).view_as(tensor))
        offset += numel
    return tuple(outputs)


def scatter_tensors(flat, tensors):
    """reset_model's copy-back loop (communicator.py:124-131) as one mx_scatter launch."""
    tensors = list(tensors)
    for t in tensors:
        if t.device != flat.device or t.dtype != torch.float32 or not t.is_contiguous():
            raise TypeError("scatter_tensors: contiguous float32 tensors on flat's CUDA device required")
    off = _offsets(tensors)
    total = int(off[-1])
    if total:
        ptrs = torch.tensor([t.data_ptr() for t in tensors], dtype=torch.int64, device=flat.device)
        offd = torch.from_numpy(off).to(flat.device)
        with torch.cuda.device(flat.device):
            check(lib.mx_scatter(ptrs.data_ptr(), offd.data_ptr(), len(tensors), total, flat.data_ptr(),
                                 stream_ptr()), "mx_scatter")


def communicate(tensors, communication_op):
    """comm_helpers.py:59-75 (unused by the reference's hot path): flatten, apply op, write back."""
    flat_tensor = flatten_tensors(tensors)
    communication_op(tensor=flat_tensor)
    for f, t in zip(unflatten_tensors(flat_tensor, tensors), tensors):
        t.set_(f)
