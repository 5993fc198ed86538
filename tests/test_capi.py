"""CPU checks of the C-ABI library: it loads, exports every symbol declared in
include/preganplus.h, and its host-side logic (blob length, argument checks)
behaves — no compute calls (no GPU here)."""
import ctypes
import re

import numpy as np
import pytest

from preganplus_amd import _native
from preganplus_amd import weights as W


def declared_symbols():
    txt = open("include/preganplus.h").read()
    return sorted(set(re.findall(r"\b(pgp_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = _native.lib()
    syms = declared_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(L, s), f"missing export {s}"


def test_every_ctypes_call_declares_argtypes():
    """Every pgp_* entry point called through ctypes has argtypes set somewhere
    in the package: without them ctypes passes Python ints as 32-bit C ints and
    silently truncates device pointers (a GPU memory fault, not an error)."""
    import glob
    files = glob.glob("preganplus_amd/*.py") + glob.glob("tools/*.py") + glob.glob("tests/*.py") + ["bench.py"]
    calls, decl = {}, set()
    for f in files:
        s = open(f).read()
        for name in re.findall(r"\.(pgp_\w+)\(", s):
            calls.setdefault(name, f)
        decl |= set(re.findall(r"\.(pgp_\w+)\.argtypes", s))
    missing = {k: v for k, v in calls.items() if k not in decl}
    assert not missing, missing


def test_abi_version_and_hosts():
    L = _native.lib()
    assert L.pgp_abi_version() == 1
    hs = _native.supported_hosts()
    assert 16 in hs and 50 in hs
    assert all(h % 2 == 0 for h in hs)


@pytest.mark.parametrize("H", [8, 16, 32, 50, 64])
def test_blob_length_matches_python_layout(H):
    L = _native.lib()
    assert L.pgp_weight_blob_len(H, H) == W.blob_size(H)
    assert L.pgp_weight_blob_len(H, 3) == W.blob_size(H, 3)


def test_shipped_weights_blob_length():
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    assert W.pack_blob(w, 16).size == _native.lib().pgp_weight_blob_len(16, 16)


def test_argument_errors():
    L = _native.lib()
    h = ctypes.c_void_p()
    assert L.pgp_create(15, 15, ctypes.byref(h)) == -2        # odd / not compiled
    assert L.pgp_create(16, 0, ctypes.byref(h)) == -1
    assert L.pgp_create(16, 16, ctypes.byref(h)) == 0
    blob = np.zeros(10)
    rc = L.pgp_load_weights(h, blob.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 10)
    assert rc == -1 and b"length" in L.pgp_last_error()
    # forward before weights -> state error, no device work
    rc = L.pgp_forward(h, 4, *([None] * 11), None)
    assert rc == -4
    assert L.pgp_destroy(h) == 0
    assert L.pgp_weight_blob_len(7, 7) == 0


def test_fpe_variant_abi():
    """PreGAN FPE variant: blob length agrees with the Python layout, host
    count and argument errors surface before any device work."""
    L = _native.lib()
    w, _ = W.load_npz("preganplus_amd/data/pregan_simulator_16.npz")
    assert W.pack_blob(w, 16).size == L.pgp_fpe_weight_blob_len(16)
    # 50 hosts: the FPE_16 code at n_hosts=50 (make_golden_fpe50.py), not the crashing FPE_50
    assert W.pack_blob(W.synth_fpe_weights(50, 0), 50).size == L.pgp_fpe_weight_blob_len(50)
    assert L.pgp_fpe_weight_blob_len(32) == 0
    h = ctypes.c_void_p()
    assert L.pgp_create_fpe(32, ctypes.byref(h)) == -2
    assert L.pgp_create_fpe(50, ctypes.byref(h)) == 0
    assert L.pgp_destroy(h) == 0
    assert L.pgp_create_fpe(16, ctypes.byref(h)) == 0
    blob = np.zeros(10)
    assert L.pgp_load_weights(h, blob.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 10) == -1
    assert b"FPE" in L.pgp_last_error()
    assert L.pgp_forward_fpe(h, 4, *([None] * 11), None) == -4   # weights not loaded
    assert L.pgp_destroy(h) == 0
