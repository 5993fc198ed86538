"""The executed-work roofline constant must match the BUILT library: the
v_mfma count per host and wave of encoder_kernel<H> in
preganplus_amd/_lib/libpreganplus.so (unbundled and disassembled offline by
tools/isa_count.py) equals roofline.ENC_MFMA_PER_HOST[H], so a K2 change that
moves the MFMA count fails here instead of silently corrupting bench.py's
`roofline.frac`."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from preganplus_amd import roofline as R  # noqa: E402

LIB = os.path.join(ROOT, "preganplus_amd", "_lib", "libpreganplus.so")


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="built library / llvm-objdump absent")
def test_encoder_mfma_count_matches_built_library():
    import isa_count
    counts = isa_count.encoder_counts(tuple(R.ENC_MFMA_PER_HOST))
    for H, n in R.ENC_MFMA_PER_HOST.items():
        assert counts[H][0] == n, f"H={H}: built library issues {counts[H][0]} MFMAs per host, roofline says {n}"


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="built library / llvm-objdump absent")
def test_encoder_split_mfma_counts_match_built_library():
    """The split feed-forward form: its fp32 MFMAs are the fp32 form's minus the
    feed-forward's (2 layers x (4 x 13 + 3 x 16) x 3 steps = 600), its bf16
    MFMAs 6 per 32-k block (2 layers x (4 x 2 + 3 x 2) x 6 x 3 steps = 504)."""
    import isa_count
    counts = isa_count.encoder_split_counts(tuple(R.ENC_SPLIT_MFMA_PER_HOST))
    for H, (f32, bf) in R.ENC_SPLIT_MFMA_PER_HOST.items():
        assert counts[H][:2] == (f32, bf), (H, counts[H])
    assert R.ENC_SPLIT_MFMA_PER_HOST[50][0] == R.ENC_MFMA_PER_HOST[50] - 2 * (4 * 13 + 3 * 16) * 3
    assert R.ENC_SPLIT_MFMA_PER_HOST[50][1] == 2 * (4 * 2 + 3 * 2) * 6 * 3


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="built library / llvm-objdump absent")
def test_tuning_kernel_mfma_counts_match_built_library():
    import isa_count
    counts = isa_count.tune_counts(tuple(R.TUNE_MFMA_PER_UNIT))
    assert counts == R.TUNE_MFMA_PER_UNIT
    bf = isa_count.tune_counts(tuple(R.TUNE_BF16_PER_UNIT), op="_f32_16x16x32_bf16")
    assert bf == R.TUNE_BF16_PER_UNIT


def test_tune_fused_flops_bookkeeping():
    # layer 1's forward = the forward kernel's count minus layer 0's time encoder
    f = R.tune_fused_flops(50, 1030)
    units = (1030 * 50 + 15) // 16
    assert f[0] - f[1] == units * R.tune_te_mfma(50) * 2048 == units * 4 * 14 * 3 * 2048
    assert f[2] == f[4] and f[3] == f[5]
    assert R.tune_te_mfma(16) == 1 * 4 * 3


def test_executed_rate_cannot_exceed_peak_definition():
    # executed flops per window are what K2 issues; the reference formulation's
    # count is reported separately as an algorithmic rate
    for H in R.ENC_MFMA_PER_HOST:
        assert R.encoder_executed_flops_per_window(H) == R.ENC_MFMA_PER_HOST[H] * 2048 * H / 16


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="built library / llvm-objdump absent")
def test_fused_tuning_prefetches_are_not_waited_for_at_once():
    """The fused tuning kernels prefetch the next unit's 12 input tiles during
    a GEMM; a value select right after the loads made the compiler wait for
    them at once (0 MFMAs of cover).  Loads outside the batch select the
    ADDRESS (pgp_tunef.hip row_ptr), so each prefetch has a GEMM's worth of
    MFMAs before its wait in the built library."""
    import isa_count
    for name in ("tf_fwd_kernel", "tf_bwd_ffn_kernel", "tf_bwd_att_kernel"):
        cover = isa_count.load_cover(name, 50)
        assert sum(1 for c in cover if c >= 48) >= 12, (name, cover)


def test_weight_gradient_and_decoder_prefetches_are_covered():
    """The token-major weight-gradient contraction (dw_accumulate: in_proj,
    time encoder, GAT fc, decoders) prefetches the next 32-row chunk while the
    current one is contracted from LDS, and the decoder forward loads the next
    token's rows under this token's MFMAs.  Zeros for rows past the range come
    from a selected ADDRESS (pgp_gemm.hpp dw_zero4), the chunk loop is
    branch-free, and dec_fwd2 reads only the live features of its last
    k-block, so no prefetch is waited for before the MFMAs it should hide
    behind (before: 24 / 16 / 0 MFMAs of cover)."""
    import isa_count
    for name, tag, need, n in (("dw_kernel", "192ELi64", 96, 8), ("dec_dw_kernel", "50", 64, 9),
                               ("dec_fwd2_kernel", "50", 128, 4)):
        cover = isa_count.load_cover(name, tag)
        assert sum(1 for c in cover if c >= need) >= n, (name, cover)


def _pmc_files():
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*_h*.json")))


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="built library / llvm-objdump absent")
def test_committed_pmc_traffic_matches_built_library():
    """Every committed PMC traffic file (profiles/pmc_<kernel>_h<H>.json, the
    source of bench.py's `traffic` fields) was taken with the kernel as it is
    built now: its isa_sha256 equals the built library's instructions of that
    kernel.  A kernel change without a new counter pass fails here (VERDICT r3
    item 1: stale r02 counters were reported as r03 traffic)."""
    import json
    import re
    import isa_count
    files = _pmc_files()
    assert files
    for f in files:
        d = json.load(open(f))
        m = re.match(r"pmc_(\w+)_h(\d+)\.json", os.path.basename(f))
        want = isa_count.kernel_isa_hash(m.group(1) + "_kernel", int(m.group(2)), targs=d.get("template_args"))
        assert d.get("isa_sha256") == want, f"{os.path.basename(f)} is stale (taken with another build)"


def test_bench_traffic_ignores_other_builds(tmp_path):
    """bench.py reports a PMC file's traffic only for the batch it was taken at
    and only when its isa_sha256 matches the loaded library's kernel."""
    import json
    import bench
    p = tmp_path / "pmc.json"
    rec = {"hbm_bytes_per_launch": 123.0, "batch": 64, "isa_sha256": "0" * 64}
    p.write_text(json.dumps(rec))
    assert bench.traffic_record(50, 64, "encoder", path=str(p)) is None       # another build
    rec["isa_sha256"] = bench.loaded_isa_hash("encoder_kernel", 50)
    if rec["isa_sha256"] is not None:
        p.write_text(json.dumps(rec))
        assert bench.traffic_record(50, 64, "encoder", path=str(p))["hbm_bytes_per_launch"] == 123.0
        assert bench.traffic_record(50, 65, "encoder", path=str(p)) is None   # another batch


@pytest.mark.skipif(not os.path.exists(LIB) or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"),
                    reason="built library / llvm-objdump absent")
def test_gobi_dpp_sources_clear_of_valu_writes():
    """GOBI's row_newbcast multiply-adds are inline asm, outside the compiler's
    hazard check: in the built gobi_kernel no VALU write of a DPP source sits
    within the 2 wait states the hardware needs (tools/dpp_hazard_check.py)."""
    import re
    import dpp_hazard_check
    import isa_count
    asm = isa_count._disasm(LIB, "gobi_kernel")
    m = re.search(r"^[0-9a-f]+ <_ZN3pgp12_GLOBAL__N_1\d+gobi_kernel[^>]*>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", asm, re.S | re.M)
    assert m is not None, "gobi_kernel not found in the built library"
    insts = dpp_hazard_check.parse(m.group(1).split("\n"))
    n, found = dpp_hazard_check.check_insts(insts)
    assert n > 100, f"only {n} DPP instructions: the row_newbcast chains are gone?"
    assert not found, found[:5]
