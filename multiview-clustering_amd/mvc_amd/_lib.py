"""ctypes binding of libmvc_hip.so (the C ABI declared in include/mvc.h).

The library is built in-tree (``make`` at the repo root ->
multiview-clustering_amd/lib/libmvc_hip.so).  There is no CPU fallback: if
the library is missing, or no HIP device is visible when a sampler is
created, the call raises.
"""
import ctypes
import os

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("MVC_HIP_LIB", os.path.join(_PKG_DIR, "lib", "libmvc_hip.so"))

MVC_OK = 0
MODE_EXACT = 0
MODE_PARALLEL = 1
FLAG_TIMING = 1
FLAG_QUIET = 2
FLAG_TIMING_COARSE = 4
TRACE_ALPHA_V, TRACE_SIGMA_V, TRACE_TAU_V, TRACE_ALPHA_GLOBAL, TRACE_SIGMA_GLOBAL = range(5)


ABI_VERSION = 2
MVC_ERR_CALLBACK = 5

# all_gather callback of mvc_sampler_set_shard: int (*)(void *user), 0 = done
SHARD_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


class MvcError(RuntimeError):
    """Error returned through the C ABI (status code + message)."""

    def __init__(self, code, msg):
        super().__init__(f"mvc error {code}: {msg}")
        self.code = code


class Config(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int32),
        ("n_views", ctypes.c_int32),
        ("dim", ctypes.c_int32),
        ("n_iter", ctypes.c_int32),
        ("burn_in", ctypes.c_int32),
        ("thin", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("n_chains", ctypes.c_int32),
        ("first_chain", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("table_cap", ctypes.c_int32),
        ("dish_cap", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("n_devices", ctypes.c_int32),      # ABI 2
        ("chain_stride", ctypes.c_int32),
    ]


_lib = None


def lib():
    """Load libmvc_hip.so (raises FileNotFoundError / OSError loudly)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(
            f"{LIB_PATH} not found: build the HIP extension first (make, or __graft_entry__.build())")
    # No hardware-queue request: a handle's chains share one stream for
    # their repair (the chain-batched repair), so HIP's default
    # of 4 queues serves them; GPU_MAX_HW_QUEUES is left as the caller set it.
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32, u64, sz = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32,
                                  ctypes.c_uint64, ctypes.c_size_t)
    cp = ctypes.c_char_p
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int32)
    lp = ctypes.POINTER(ctypes.c_int64)
    cfgp = ctypes.POINTER(Config)
    vpp = ctypes.POINTER(vp)
    sig = {
        "mvc_config_init": (None, [cfgp]),
        "mvc_abi_version": (i32, []),
        "mvc_last_error": (cp, []),
        "mvc_run": (i32, [cfgp, ctypes.POINTER(dp), vpp, cp, sz]),
        "mvc_result_num_saved": (i32, [vp]),
        "mvc_result_num_chains": (i32, [vp]),
        "mvc_result_num_tables": (i32, [vp, i32, i32]),
        "mvc_result_table_of": (ip, [vp, i32, i32]),
        "mvc_result_dish_of": (ip, [vp, i32, i32]),
        "mvc_result_trace": (dp, [vp, i32, i32]),
        "mvc_result_copy_chain": (i32, [vp, i32, ip, ip, ip]),
        "mvc_result_summary": (i32, [vp, dp, dp]),
        "mvc_result_free": (None, [vp]),
        "mvc_sampler_create": (i32, [cfgp, ctypes.POINTER(dp), vpp, cp, sz]),
        "mvc_sampler_sweep": (i32, [vp, i32, cp, sz]),
        "mvc_sampler_synchronize": (i32, [vp, cp, sz]),
        "mvc_sampler_sweeps_done": (i32, [vp]),
        "mvc_sampler_get_state": (i32, [vp, i32, ip, ip, ip, ctypes.c_int32, dp, cp, sz]),
        "mvc_sampler_get_dish_counts": (i32, [vp, i32, ip, cp, sz]),
        "mvc_sampler_set_state": (i32, [vp, i32, ip, ctypes.c_int32, ip, dp, cp, sz]),
        "mvc_sampler_get_stats": (i32, [vp, i32, i32, ip, dp, dp, ip, ctypes.c_int32, cp, sz]),
        "mvc_sampler_kernel_time": (i32, [vp, cp, dp, lp]),
        "mvc_sampler_reset_timers": (None, [vp]),
        "mvc_sampler_zpath": (i32, [vp]),
        "mvc_sampler_repair_stats": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int32)]),
        "mvc_sampler_phase_a": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int32)]),
        "mvc_sampler_set_timing": (i32, [vp, i32]),
        "mvc_sampler_ari": (i32, [vp, i32, ip, dp, cp, sz]),
        "mvc_ari": (i32, [i32, ip, ip, i64, dp, cp, sz]),
        "mvc_sampler_stream": (vp, [vp]),
        "mvc_sampler_create_synthetic": (i32, [cfgp, ctypes.c_int32, u64, ctypes.c_double, ctypes.c_double, ip, vpp,
                                               cp, sz]),
        "mvc_sampler_copy_rows": (i32, [vp, ctypes.c_int32, ip, i64, dp, cp, sz]),
        "mvc_sampler_set_shard": (i32, [vp, i32, i32, vp, vp, vp]),
        "mvc_shard_len": (i64, [i64, i32]),
        "mvc_sampler_destroy": (None, [vp]),
        "mvc_device_math": (i32, [i32, i32, dp, dp, i64, cp, sz]),
        "mvc_device_seq_uniforms": (i32, [i32, u64, u32, u64, dp, i64, cp, sz]),
        "mvc_device_tree64": (i32, [i32, dp, i64, i64, dp, dp, lp, cp, sz]),
        "mvc_device_gemm_check": (i32, [i32, dp, dp, i64, i64, i64, dp, cp, sz]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.mvc_abi_version() != ABI_VERSION:
        raise OSError(f"{LIB_PATH}: ABI version {L.mvc_abi_version()}, this binding needs {ABI_VERSION}")
    _lib = L
    return L


def errbuf():
    return ctypes.create_string_buffer(1024)


def check(status, buf):
    if status != MVC_OK:
        raise MvcError(status, buf.value.decode(errors="replace"))
