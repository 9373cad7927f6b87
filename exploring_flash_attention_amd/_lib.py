"""ctypes binding of libfa_mi355x.so (the C ABI declared in include/fa_mi355x.h).

The library is built in-tree by ``python __graft_entry__.py`` (or ``make -C
exploring_flash_attention_amd/csrc``) and loaded from ``exploring_flash_attention_amd/_lib/``.
There is no fallback: if the library is missing, ``lib()`` raises.
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FA_MI355X_LIB", os.path.join(_HERE, "_lib", "libfa_mi355x.so"))

FA_OK = 0
FA_ERR_INVALID_ARG = 1
FA_ERR_UNSUPPORTED = 2
FA_ERR_HIP = 3
FA_ERR_WORKSPACE = 4

FA_DTYPE_FP16 = 0
FA_DTYPE_BF16 = 1
FA_DTYPE_FP32 = 2
FA_DTYPE_FP64 = 3
FA_DTYPE_FP16_SCALED = 4  # split-KV partials: fp16 scaled per row by a power of two

FA_KV_TILES_AUTO = -1  # kv_tiles_per_block: split chosen from the device's occupancy
FA_BLOCKS_PER_WG_AUTO = 0  # blocks_per_workgroup: the library groups the key blocks itself
FA_V2_COUNTERS_ZERO = 1  # fa_fwd_v2_ex2: the caller vouches that the workspace counters are zero

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I = ctypes.c_int
_PI = ctypes.POINTER(ctypes.c_int)

# name -> (restype, argtypes); must cover every function in include/fa_mi355x.h
SIGNATURES = {
    "fa_version": (_I, []),
    "fa_last_error": (ctypes.c_char_p, []),
    "fa_last_kernels": (ctypes.c_char_p, []),
    "fa_kernel_geometry": (_I, [_I64, _I, ctypes.POINTER(_I), ctypes.POINTER(_I),
                                ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "fa_fwd_v1": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _P]),
    "fa_fwd_v1_scaled": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, ctypes.c_double, _I, _P]),
    "fa_fwd_v1_ex": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _P, _P, _P, ctypes.c_double, _I, _P]),
    "fa_fwd_v1_tiled_d": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _I, _I, _P]),
    "fa_fwd_v1_tiled_d_scaled": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _I, ctypes.c_double, _I, _P]),
    "fa_fwd_v2_split_plan": (_I, [_I64, _I64, _I64, _I64, _I, _I, _I, _PI, _PI, _PI]),
    "fa_fwd_v2_workspace_size": (_I, [_I64, _I64, _I64, _I64, _I, _I, _I,
                                      ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_I)]),
    "fa_fwd_v2_workspace_size_ex": (_I, [_I64, _I64, _I64, _I64, _I, _I, _I, _I,
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(_I)]),
    "fa_fwd_v2": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _I, _I, _P, ctypes.c_size_t,
                       _I, _I, _P]),
    "fa_fwd_v2_scaled": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _I, _I, _P, ctypes.c_size_t,
                              ctypes.c_double, _I, _I, _P]),
    "fa_fwd_v2_ex": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _I, _I, _I, _P, ctypes.c_size_t,
                          _P, _P, _P, ctypes.c_double, _I, _I, _P]),
    "fa_fwd_v2_ex2": (_I, [_P, _P, _P, _P, _I64, _I64, _I64, _I64, _I, _I, _I, _I, _P, ctypes.c_size_t,
                           _P, _P, _P, ctypes.c_double, _I, _I, ctypes.c_uint, _P]),
    "fa_fwd_partial": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _I, _I, _P]),
    "fa_fwd_partial_ex": (_I, [_P, _P, _P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I64, _P, _I, _I, _P]),
    "fa_combine": (_I, [_P, _P, _P, _I64, _I64, _I64, _I64, _I64, _I, _I, _P]),
}

_lock = threading.Lock()
_lib = None


class FaError(RuntimeError):
    """A non-FA_OK status from the C ABI."""

    def __init__(self, status, message):
        super().__init__(f"[fa status {status}] {message}")
        self.status = status


class FaArgumentError(FaError, ValueError):
    """FA_ERR_INVALID_ARG / FA_ERR_UNSUPPORTED / FA_ERR_WORKSPACE."""


def lib():
    """Load (once) and return the ctypes handle; raise if the library is not built."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"{LIB_PATH} is missing: build it with `python __graft_entry__.py` "
                        "(hipcc --offload-arch=gfx950); there is no CPU fallback")
                h = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    fn = getattr(h, name)
                    fn.restype = res
                    fn.argtypes = args
                _lib = h
    return _lib


def check(status):
    """Raise FaArgumentError / FaError for a non-zero status."""
    if status == FA_OK:
        return
    msg = lib().fa_last_error().decode(errors="replace")
    if status in (FA_ERR_INVALID_ARG, FA_ERR_UNSUPPORTED, FA_ERR_WORKSPACE):
        raise FaArgumentError(status, msg)
    raise FaError(status, msg)


def last_kernels():
    """The kernels (with their grids) the last launching C-ABI call of this thread enqueued,
    as the library's launcher chose them (fa_last_kernels)."""
    return lib().fa_last_kernels().decode(errors="replace")


def geometry(d, dtype=FA_DTYPE_BF16):
    """(bq, bk, threads, lds_bytes) of the forward kernel for head dim d."""
    vals = [_I() for _ in range(4)]
    check(lib().fa_kernel_geometry(d, dtype, *[ctypes.byref(v) for v in vals]))
    return tuple(v.value for v in vals)
