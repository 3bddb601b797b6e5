"""ctypes binding of libba3c.so (include/ba3c.h).  No fallback: if the HIP library is
missing or fails to load, every product entry point raises Ba3cLibraryError."""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# BA3C_LIB: an alternative in-tree build of the same ABI (A/B experiments, scripts/gpu_abl.sh)
LIB_PATH = os.environ.get("BA3C_LIB") or os.path.join(_HERE, "libba3c.so")

BA3C_OK = 0
OPT_IDS = {"adam": 0, "gd": 1, "adagrad": 2, "adadelta": 3, "momentum": 4, "rms": 5}
SCALAR_NAMES = ["cost", "policy_loss", "xentropy_loss", "value_loss", "advantage",
                "pred_reward", "max_logit", "active_relus"]
KERNEL_IDS = {
    "conv0_fwd": 0, "conv1_fwd": 1, "conv2_fwd": 2, "conv3_fwd": 3, "fc1_fwd": 4, "heads": 5,
    "fc1_dgrad": 6, "conv3_dgrad": 7, "conv2_dgrad": 8, "conv1_dgrad": 9, "head_wgrad": 10,
    "fc1_wgrad": 11, "conv3_wgrad": 12, "conv2_wgrad": 13, "conv1_wgrad": 14, "conv0_wgrad": 15,
    "wgrad_reduce": 16, "clip": 17, "update": 18, "scalars": 19,
}


class Ba3cLibraryError(RuntimeError):
    pass


class Ba3cConfig(ctypes.Structure):
    _fields_ = [("max_batch", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("fc_neurons", ctypes.c_int32), ("fc_splits", ctypes.c_int32),
                ("num_actions", ctypes.c_int32), ("replace_with_conv", ctypes.c_int32),
                ("ps", ctypes.c_int32)]


class Ba3cOptParams(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("epsilon", ctypes.c_float), ("beta1_power", ctypes.c_float),
                ("beta2_power", ctypes.c_float), ("decay", ctypes.c_float),
                ("momentum", ctypes.c_float), ("rho", ctypes.c_float)]


_lib = None
# roofline-accounting queries an alternative A/B build (BA3C_LIB) may predate
AB_OPTIONAL = {"ba3c_kernel_merged", "ba3c_probe_every"}


def load():
    """Load libba3c.so once and declare every prototype of include/ba3c.h."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Ba3cLibraryError(
            "libba3c.so not found at %s — build it with `make -C distributed-ba3c_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback" % LIB_PATH)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:
        raise Ba3cLibraryError("failed to load %s: %s" % (LIB_PATH, e))
    P, i32, i64, f32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
    sig = {
        "ba3c_version": (i32, []),
        "ba3c_last_error": (ctypes.c_char_p, []),
        "ba3c_create": (i32, [ctypes.POINTER(Ba3cConfig), ctypes.POINTER(P)]),
        "ba3c_destroy": (None, [P]),
        "ba3c_num_tensors": (i32, [P]),
        "ba3c_tensor_info": (i32, [P, i32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(i64),
                                   ctypes.POINTER(i64), ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "ba3c_flat_size": (i64, [P]),
        "ba3c_workspace_size": (ctypes.c_size_t, [P, i32, i32]),
        "ba3c_workspace_tensor": (i32, [P, i32, i32, ctypes.c_char_p, ctypes.POINTER(i64),
                                        ctypes.POINTER(i64)]),
        "ba3c_forward": (i32, [P, P, P, P, i32, f32, P, P, P, P]),
        "ba3c_train_grads": (i32, [P, P, P, P, P, P, i32, f32, P, P, P]),
        "ba3c_clip_grads": (i32, [P, P, P, P]),
        "ba3c_clip_grads_range": (i32, [P, P, P, P, i32, i32]),
        "ba3c_train_grads_phase": (i32, [P, P, P, P, P, P, i32, f32, P, P, P, i32]),
        "ba3c_bucket_tensor": (i32, [P]),
        "ba3c_flush_pending": (i32, [P]),
        "ba3c_launch_held": (i32, [P, P]),
        "ba3c_set_phase2_event": (i32, [P, P]),
        "ba3c_clip_grads_range2": (i32, [P, P, P, P, i32, i32, i32]),
        "ba3c_occupy_cus": (i32, [P, i32, ctypes.c_double]),
        "ba3c_comm_unique_id": (i32, [P]),
        "ba3c_comm_init": (i32, [P, P, i32, i32]),
        "ba3c_comm_destroy": (i32, [P, i32]),
        "ba3c_allreduce_sum": (i32, [P, P, P, i64]),
        "ba3c_allreduce_mean": (i32, [P, P, P, i64]),
        "ba3c_apply_update": (i32, [P, P, i32, P, P, P, P, ctypes.POINTER(Ba3cOptParams), f32,
                                    i32, P]),
        "ba3c_apply_update_dev": (i32, [P, P, i32, P, P, P, P, ctypes.POINTER(Ba3cOptParams), P,
                                        f32, i32, P]),
        "ba3c_sample": (i32, [P, P, P, i32, i32, P, P]),
        "ba3c_greedy": (i32, [P, P, P, P, i32, i32, ctypes.c_double, P]),
        "ba3c_probe_enable": (i32, [P, i32]),
        "ba3c_probe_every": (i32, [P, i32]),
        "ba3c_probe_read": (i32, [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i32)]),
        "ba3c_device_errors": (i32, [P, ctypes.POINTER(ctypes.c_uint32)]),
        "ba3c_kernel_split": (i32, [P, i32]),
        "ba3c_kernel_merged": (i32, [P, i32]),
        "ba3c_kernel_family": (i32, [P, i32]),
        "ba3c_nstep_returns": (i32, [P, P, P, P, P, P, i32, i32, ctypes.c_double, P, P, P, P, P]),
        "ba3c_gather_rows": (i32, [P, P, P, i32, i64, P]),
        "ba3c_history_push": (i32, [P, P, P, P, i32, i32, i32, i32]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("BA3C_LIB") and name in AB_OPTIONAL and not hasattr(lib, name):
            continue            # an A/B build older than this accounting query
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status):
    if status != BA3C_OK:
        msg = _lib.ba3c_last_error().decode() if _lib is not None else "?"
        raise Ba3cLibraryError("libba3c error %d: %s" % (status, msg))
