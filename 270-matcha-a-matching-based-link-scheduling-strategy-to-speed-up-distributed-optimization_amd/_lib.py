"""ctypes binding of the gfx950 C ABI (include/matcha_gossip.h -> _native/libmatcha_gossip.so).

There is no fallback: if the library is missing the package import fails loudly, and every
compute entry point needs a HIP device.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MX_GOSSIP_LIB: another build of the same library (A/B timing of kernel variants in one run)
LIB_PATH = os.environ.get("MX_GOSSIP_LIB") or os.path.join(_HERE, "_native", "libmatcha_gossip.so")

c_int, c_i64, c_u64, c_f32, c_f64 = ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_double
c_p = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/matcha_gossip.h one to one
SIGNATURES = {
    "mx_version": (ctypes.c_char_p, []),
    "mx_last_error": (ctypes.c_char_p, []),
    "mx_flags_binomial": (c_int, [c_p, c_int, c_p, c_int, c_i64, c_p, c_p, c_p, c_p]),
    "mx_flags_binomial_sequential": (c_int, [c_p, c_int, c_p, c_int, c_i64, c_p, c_p, c_p, c_p]),
    "mx_plan_words": (c_i64, [c_int, c_int]),
    "mx_plan_build": (c_int, [c_p, c_i64, c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_f64, c_p, c_p]),
    "mx_plan_set_idle": (c_int, [c_p, c_i64, c_int, c_int, c_int, c_p]),
    "mx_mix_tile": (c_int, [c_int]),
    "mx_mix_layout": (c_int, [c_p, c_int, c_int, c_p]),
    "mx_mix_set": (c_int, [ctypes.c_char_p, c_int]),
    "mx_mix_get": (c_int, [ctypes.c_char_p]),
    "mx_mix_kernel_name": (ctypes.c_char_p, [c_int]),
    "mx_gossip_mix": (c_int, [c_p, c_p, c_p, c_p, c_int, c_i64, c_int, c_p, c_i64, c_int, c_int, c_f32, c_p]),
    "mx_gossip_mix_packed": (c_int, [c_p, c_i64, c_p]),
    "mx_gossip_mix_at": (c_int, [c_p, c_p, c_p, c_p, c_int, c_i64, c_int, c_p, c_p, c_i64, c_int, c_int, c_f32,
                                 c_p]),
    "mx_iter_advance": (c_int, [c_p, c_i64, c_p]),
    "mx_gather": (c_int, [c_p, c_p, c_int, c_i64, c_p, c_p]),
    "mx_scatter": (c_int, [c_p, c_p, c_int, c_i64, c_p, c_p]),
    "mx_topk_work_bytes": (ctypes.c_size_t, [c_i64]),
    "mx_iter_expand": (c_int, [c_p, c_p, c_int, c_p]),
    "mx_topk_set": (c_int, [ctypes.c_char_p, c_i64]),
    "mx_topk_get": (c_i64, [ctypes.c_char_p]),
    "mx_topk_check": (c_int, [c_p, c_i64, c_int, c_i64, c_p]),
    "mx_topk_err_forward": (c_int, [c_p, c_i64, c_int, c_i64, c_p, c_p]),
    "mx_topk_stats": (c_int, [c_p, c_i64, c_int, c_i64, c_p, c_p]),
    "mx_topk_trace": (c_int, [c_p, c_i64]),
    "mx_topk_abs_diff": (c_int, [c_p, c_p, c_i64, c_i64, c_p, c_p, c_p, c_p]),
    "mx_topk_abs_diff_rows": (c_int, [c_p, c_p, c_i64, c_int, c_i64, c_i64, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_p]),
    "mx_choco_msg_bytes": (c_i64, [c_i64, c_i64]),
    "mx_choco_apply_work_bytes": (ctypes.c_size_t, [c_i64, c_int]),
    "mx_choco_apply": (c_int, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_int, c_p, c_i64, c_int,
                               c_int, c_f32, c_f32, c_p, c_p]),
    "mx_choco_apply_at": (c_int, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_i64, c_int, c_p, c_p, c_i64, c_int,
                                  c_int, c_f32, c_f32, c_p, c_p]),
    "mx_pull_fetch": (c_int, [c_p, c_int, c_int, c_p, c_p, c_i64, c_i64, c_p]),
    "mx_choco_apply_slots": (c_int, [c_p, c_p, c_p, c_i64, c_i64, c_i64, c_p, c_int, c_p, c_i64, c_int, c_int,
                                     c_f32, c_f32, c_p]),
    "mx_rccl_unique_id": (c_int, [c_p]),
    "mx_rccl_init": (c_int, [c_p, c_int, c_int, c_p]),
    "mx_rccl_init_timeout": (c_int, [c_p, c_int, c_int, c_i64, c_p, c_p]),
    "mx_rccl_abort": (c_int, [c_p]),
    "mx_rccl_destroy": (c_int, [c_p]),
    "mx_rccl_count": (c_int, [c_p, c_p]),
    "mx_rccl_wait": (c_int, [c_p, c_p, c_i64]),
    "mx_exchange_plan": (c_int, [c_p, c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_p, c_int, c_p]),
    "mx_exchange_post": (c_int, [c_p, c_p, c_int, c_p, c_int, c_p, c_i64, c_i64, c_p]),
    "mx_exchange_round": (c_int, [c_p, c_p, c_int, c_p, c_int, c_p, c_int, c_int, c_int, c_p, c_p, c_i64,
                                  c_i64, c_p, c_p]),
    "mx_allreduce_mean": (c_int, [c_p, c_p, c_i64, c_int, c_p]),
    "mx_allreduce_mean_ordered": (c_int, [c_p, c_p, c_i64, c_p, c_int, c_p]),
    "mx_allgather": (c_int, [c_p, c_p, c_i64, c_p, c_p]),
    "mx_mean_rows": (c_int, [c_p, c_int, c_i64, c_i64, c_int, c_p, c_p]),
    "mx_mean_rows_to": (c_int, [c_p, c_int, c_i64, c_i64, c_int, c_p, c_int, c_i64, c_p]),
    "mx_mean_kernel_name": (ctypes.c_char_p, [c_p, c_int, c_i64, c_i64, c_int, c_p, c_int, c_i64]),
    "mx_pull_gate": (c_int, [c_p, c_p, c_int, c_p, c_int, c_p, c_p, c_int, c_int, c_int, c_int, c_i64, c_int, c_u64,
                             c_p, c_int, c_f64, c_p, c_p]),
    "mx_host_words": (c_int, [c_int, c_p, c_p]),
    "mx_host_words_free": (c_int, [c_p]),
    "mx_synth_fill": (c_int, [c_p, c_i64, c_u64, c_p]),
    "mx_max_weight_matching": (c_int, [c_int, c_p, c_p, c_p, c_int, c_p, c_p, c_p]),
    "mx_snapshot_publish": (c_int, [c_p, c_p, c_i64, c_p]),
    "mx_snapshot_publish_rows": (c_int, [c_p, c_i64, c_p, c_i64, c_i64, c_int, c_p, c_int, c_p, c_int, c_int, c_p]),
    "mx_plan_set_peer_reads": (c_int, [c_p, c_i64, c_int, c_int, c_int, c_p]),
    "mx_ipc_handle_bytes": (c_int, []),
    "mx_ipc_alloc": (c_int, [c_i64, c_p, c_p]),
    "mx_ipc_stats": (c_int, [c_p, c_p]),
    "mx_ipc_set": (c_int, [ctypes.c_char_p, c_i64]),
    "mx_ipc_get": (c_i64, [ctypes.c_char_p]),
    "mx_ipc_open": (c_int, [c_p, c_p]),
    "mx_ipc_close": (c_int, [c_p]),
    "mx_ipc_free": (c_int, [c_p]),
}


MX_OK, MX_ERR_INVALID, MX_ERR_HIP, MX_ERR_RCCL, MX_ERR_RNG, MX_ERR_UNSUPPORTED = 0, -1, -2, -3, -4, -5


class MXError(RuntimeError):
    """A negative status from the native library (message from mx_last_error)."""


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"native gossip library not built: {LIB_PATH} is missing. Build it with "
            f"`make -C {_HERE}` (hipcc --offload-arch=gfx950) or __graft_entry__.build().")
    # torch first: it brings its own libamdhip64.so.7 / librccl / libhsa-runtime64 (same SONAMEs as
    # /opt/rocm's), and the loader then binds this library to those already-loaded objects, so the
    # process has ONE HIP runtime whose device pointers and streams both sides share.  Loading
    # this library first would pull /opt/rocm's runtime in under torch's feet.
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()


def check(rc, what=""):
    if rc != 0:
        msg = lib.mx_last_error().decode(errors="replace")
        raise MXError(f"{what or 'matcha-gossip'} failed ({rc}): {msg}")
    return rc


def stream_ptr(stream=None):
    """hipStream_t of a torch stream (default: torch's current stream on the current device).
    The default is read as a raw handle (no torch.cuda.Stream object is built): a small-row round
    is launch-bound, and building that object cost about as much as the kernel launch."""
    if stream is not None:
        return stream.cuda_stream
    return _raw_stream(_cur_dev())


def _bind_stream_getters():
    import torch
    return torch._C._cuda_getCurrentRawStream, torch._C._cuda_getDevice


_raw_stream, _cur_dev = _bind_stream_getters()


def require_device():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError(
            "matcha-gossip runs on an MI355X (gfx950) GPU; no HIP device is visible. There is "
            "no CPU path.")
