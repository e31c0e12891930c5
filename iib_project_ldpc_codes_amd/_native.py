"""ctypes binding of libldpc_mi355x.so (C ABI: include/ldpc_mi355x.h).

The library is the only compute path.  There is no CPU fallback: when the
shared object is missing or no MI355X is visible the calls raise
:class:`LdpcError`.
"""
import ctypes as ct
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# LDPC_LIB_PATH: benchmark another build of the library (scripts/bench_bec.py --compare)
LIB_PATH = os.environ.get("LDPC_LIB_PATH") or os.path.join(HERE, "libldpc_mi355x.so")

LDPC_OK = 0
LDPC_EINVAL, LDPC_ENODEV, LDPC_EHIP, LDPC_ENOMEM, LDPC_EUNSUP = -1, -2, -3, -4, -5
CH_BEC, CH_BSC, CH_AWGN = 0, 1, 2
ALGO_SPA, ALGO_MINSUM = 0, 1
MC_NCOUNT = 4

_lib = None


class LdpcError(RuntimeError):
    def __init__(self, func, rc, msg):
        super().__init__(f"{func} failed ({rc}): {msg}")
        self.rc = rc


def _load():
    if not os.path.exists(LIB_PATH):
        raise LdpcError("load", LDPC_ENODEV,
                        f"{LIB_PATH} not built: run `make -C iib_project_ldpc_codes_amd/csrc` "
                        "(or __graft_entry__.build())")
    # Share torch's HIP runtime when torch is present: device pointers from torch
    # tensors must be valid in the runtime this library uses (same soname,
    # libamdhip64.so.7, so the loader binds one copy).
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover
        pass
    return ct.CDLL(LIB_PATH, mode=ct.RTLD_GLOBAL)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    L = _load()
    P, i, f, u64, i64 = ct.c_void_p, ct.c_int, ct.c_float, ct.c_uint64, ct.c_int64
    sig = {
        "message_passing": ([P, i, P, P, P, i, i, i, i], i),
        "ldpc_graph_create": ([P, P, i, i, i, i, ct.POINTER(P)], i),
        "ldpc_graph_create_csr": ([P, P, P, P, i, i, ct.POINTER(P)], i),
        "ldpc_graph_destroy": ([P], None),
        "ldpc_graph_info": ([P, P, P, P], i),
        "ldpc_bec_decode_batch": ([P, P, i, i, i, i, P, i, i, P, P], i),
        "ldpc_bec_decode_batch_dev": ([P, P, i, i, P, P, P], i),
        "ldpc_bp_decode_batch": ([P, P, i, i, i, i, P, i, i, i, f, i, P, P, P], i),
        "ldpc_bp_decode_batch_dev": ([P, P, i, i, i, f, i, P, P, P, P], i),
        "ldpc_channel_dev": ([i, f, u64, u64, i, i, P, P], i),
        "ldpc_mc_batch_dev": ([P, i, f, u64, u64, i, i, i, f, i, i, i64, P, P], i),
        "ldpc_last_error": ([], ct.c_char_p),
        "ldpc_device_count": ([], i),
        "ldpc_set_device": ([i], i),
        "ldpc_sync": ([P], i),
        "ldpc_bp_kernel_name": ([P, i], ct.c_char_p),
        "ldpc_debug_lane_layout": ([P, P, i, i, i, i, P, P, P, P], i),
        "ldpc_debug_irr_layout": ([P, P, P, P, i, i, P, P, P], i),
        "ldpc_debug_loc_layout": ([P, P, P, P, i, i, i, P, P, P, P], i),
        "ldpc_debug_loc_variant": ([P, P, P, P, i, i, i, P], i),
        "ldpc_debug_mc_plan": ([P, i64, i64, i64, i, i, P], i),
        "ldpc_debug_seq_stats": ([P, i], i),
        "ldpc_debug_peel_stats": ([P, i], i),
        "ldpc_debug_peel_cap": ([i], i),
        "ldpc_sample_regular_dev": ([i, i, i, u64, u64, i, P, P, P, P], i),
        "ldpc_sample_regular": ([i, i, i, u64, u64, i, P, P, P], i),
        "ldpc_mc_ensemble_batch_dev": ([i, i, i, i, f, u64, u64, i, i, i, i64, P, P], i),
        "ldpc_sample_csr_dev": ([i, i, P, P, u64, u64, i, P, P, P, P], i),
        "ldpc_sample_csr": ([i, i, P, P, u64, u64, i, P, P, P], i),
        "ldpc_ml_decode_batch_dev": ([P, P, i, P, P, P], i),
        "ldpc_ml_decode_batch": ([P, P, i, P, P], i),
        "ldpc_ml_ensemble_decode_dev": ([i, i, i, P, P, i, P, P, P], i),
        "ldpc_mc_ml_batch_dev": ([P, i, i, i, f, u64, u64, i, i, i, i, i64, P, P, P], i),
        "ldpc_mc_run": ([P, P, i, i, i, i, i, f, i, f, i, u64, i, i, i64, i64, i, ct.c_double, P, i, P, P], i),
        "ldpc_mc_run_csr": ([P, P, P, P, i, i, i, f, i, f, i, u64, i, i, i64, i64, i, ct.c_double, P, i, P, P], i),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc, func):
    if rc is not None and rc < 0:
        raise LdpcError(func, rc, lib().ldpc_last_error().decode(errors="replace"))
    return rc


def last_error():
    return lib().ldpc_last_error().decode(errors="replace")


def exported_symbols():
    """Names the C ABI header declares (tests check they all resolve)."""
    return ["message_passing", "ldpc_graph_create", "ldpc_graph_create_csr", "ldpc_graph_destroy",
            "ldpc_graph_info", "ldpc_bec_decode_batch", "ldpc_bec_decode_batch_dev", "ldpc_bp_decode_batch",
            "ldpc_bp_decode_batch_dev", "ldpc_channel_dev", "ldpc_mc_batch_dev", "ldpc_last_error",
            "ldpc_device_count", "ldpc_set_device", "ldpc_sync", "ldpc_debug_lane_layout", "ldpc_debug_irr_layout", "ldpc_debug_loc_layout", "ldpc_bp_kernel_name", "ldpc_sample_regular_dev",
            "ldpc_sample_regular", "ldpc_mc_ensemble_batch_dev", "ldpc_ml_decode_batch_dev", "ldpc_ml_decode_batch",
            "ldpc_ml_ensemble_decode_dev", "ldpc_mc_ml_batch_dev", "ldpc_sample_csr_dev", "ldpc_sample_csr",
            "ldpc_mc_run", "ldpc_mc_run_csr", "ldpc_debug_loc_variant", "ldpc_debug_mc_plan",
            "ldpc_debug_seq_stats", "ldpc_debug_peel_stats", "ldpc_debug_peel_cap"]
