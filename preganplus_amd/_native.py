"""ctypes binding of the C-ABI in ``include/preganplus.h``.

This is the binding a maintainer of the reference would add:
the reference's interface for this path is Python, so the FFI is ctypes.
There is no fallback: if the HIP library is missing, importing the product
path raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PGP_LIB", os.path.join(_HERE, "_lib", "libpreganplus.so"))

PGP_OK = 0
_ERRS = {-1: "PGP_ERR_ARG", -2: "PGP_ERR_UNSUPPORTED", -3: "PGP_ERR_HIP", -4: "PGP_ERR_STATE"}

_lib = None

# A/B switches removed in round 5: the library and the
# Python host read none of them any more.  Setting one warns instead of
# silently measuring the default; PGP_INIT_SEED became the recoveries'
# ``init_seed`` argument.
REMOVED_ENV = ("PGP_TUNE_SIDE_STREAM", "PGP_TUNE_SIDE_MIN_TOKENS", "PGP_TUNE_DEC_DWS", "PGP_TUNE_SIDE_EARLY",
               "PGP_TUNE_EARLY_FLUSH", "PGP_TF_SPREAD", "PGP_C3_GAN_LATE", "PGP_INIT_SEED", "PGP_SAVE_GAN_INTERVAL")


def _warn_removed_env():
    import warnings
    for k in REMOVED_ENV:
        if k in os.environ:
            hint = " (use the init_seed argument)" if k == "PGP_INIT_SEED" else ""
            warnings.warn(f"{k} is no longer read by preganplus_amd{hint}; it has no effect", RuntimeWarning,
                          stacklevel=3)


class NativeError(RuntimeError):
    pass


def lib():
    """Load libpreganplus.so (built by ``make`` / ``__graft_entry__.build()``)."""
    global _lib
    if _lib is not None:
        return _lib
    _warn_removed_env()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"HIP library not found at {LIB_PATH}; build it with `make` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    c_int, c_size, vp = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p
    fp = ctypes.c_void_p  # device pointers passed as integers
    # every entry point gets argtypes: without them ctypes passes Python ints as
    # 32-bit C ints and silently truncates device pointers
    L.pgp_abi_version.argtypes = []
    L.pgp_abi_version.restype = c_int
    L.pgp_last_error.argtypes = []
    L.pgp_last_error.restype = ctypes.c_char_p
    L.pgp_supported_hosts.argtypes = [ctypes.POINTER(c_int), c_int]
    L.pgp_supported_hosts.restype = c_int
    L.pgp_weight_blob_len.argtypes = [c_int, c_int]
    L.pgp_weight_blob_len.restype = c_size
    L.pgp_create.argtypes = [c_int, c_int, ctypes.POINTER(vp)]
    L.pgp_create.restype = c_int
    L.pgp_destroy.argtypes = [vp]
    L.pgp_destroy.restype = c_int
    L.pgp_load_weights.argtypes = [vp, ctypes.POINTER(ctypes.c_double), c_size]
    L.pgp_load_weights.restype = c_int
    L.pgp_reserve.argtypes = [vp, c_int]
    L.pgp_reserve.restype = c_int
    L.pgp_forward.argtypes = [vp, c_int] + [fp] * 11 + [vp]
    L.pgp_forward.restype = c_int
    L.pgp_forward_stage.argtypes = [vp, c_int, c_int] + [fp] * 11 + [vp]
    L.pgp_forward_stage.restype = c_int
    L.pgp_create_fpe.argtypes = [c_int, ctypes.POINTER(vp)]
    L.pgp_create_fpe.restype = c_int
    L.pgp_fpe_weight_blob_len.argtypes = [c_int]
    L.pgp_fpe_weight_blob_len.restype = c_size
    L.pgp_forward_fpe.argtypes = [vp, c_int] + [fp] * 11 + [vp]
    L.pgp_forward_fpe.restype = c_int
    L.pgp_forward_fpe_stage.argtypes = [vp, c_int, c_int] + [fp] * 11 + [vp]
    L.pgp_forward_fpe_stage.restype = c_int
    L.pgp_migrations.argtypes = [c_int, c_int] + [fp] * 5 + [vp]
    L.pgp_migrations.restype = c_int
    L.pgp_embedding.argtypes = [c_int, c_int] + [fp] * 3 + [vp]
    L.pgp_embedding.restype = c_int
    L.pgp_decoder_split.argtypes = [vp, c_int]
    L.pgp_decoder_split.restype = c_int
    L.pgp_encoder_split.argtypes = [vp, c_int]
    L.pgp_encoder_split.restype = c_int
    L.pgp_gan_split.argtypes = [vp, c_int]
    L.pgp_gan_split.restype = c_int
    L.pgp_schedule_onehot.argtypes = [c_int, c_int, fp, fp, vp]
    L.pgp_schedule_onehot.restype = c_int
    _lib = L
    return L


def check(rc, what=""):
    if rc != PGP_OK:
        msg = lib().pgp_last_error().decode(errors="replace")
        raise NativeError(f"{what}: {_ERRS.get(rc, rc)}: {msg}")


def supported_hosts():
    buf = (ctypes.c_int * 16)()
    n = lib().pgp_supported_hosts(buf, 16)
    return [buf[i] for i in range(n)]
