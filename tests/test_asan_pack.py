"""The weight packer (pgp_pack.cpp + pgp_packcore.hpp, the host code behind
pgp_load_weights) under AddressSanitizer + UBSan (`make asan`): every compiled
host count, K = 3 and K = H, the FPE variant and the length-mismatch error
paths.  Host code only (GPU sanitizers are unavailable on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="no host toolchain")
def test_packer_clean_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "asan"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.count(": ok") == 12, r.stdout
