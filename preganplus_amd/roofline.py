"""Algorithmic work of the decision path, per window.

FLOPs are 2 x the multiply-accumulates of the model's dense products, counted
on the reference's formulation (unfused, unpadded: what the math requires, not
what a kernel executes).  Bytes are the compulsory HBM I/O of the path
(window + dense schedule in; logits, protos, class, target,
probs out).
"""
from __future__ import annotations

PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (VALU = f32 MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (no sparsity), MI355X_MICROARCH.md

W = 3
FF = 64
GAN_HIDDEN = 64


def macs_per_window(H: int) -> dict:
    d = H
    tokens = W * H
    hd = d // 2
    gat = tokens * 3 * d + 2 * tokens * d + W * H * H * d     # fc, decomposed scores, aggregation
    te = tokens * d * d
    per_token_layer = 3 * d * d + d * d + 2 * (W * hd) * 2 + 2 * FF * d  # qkv, out, q.k + p.v (2 heads), ffn
    layers = 2 * tokens * per_token_layer
    dec = (W * H * d) * (4 * H)                                 # anomaly + prototype decoders
    gan = GAN_HIDDEN * (2 * H + H * H) + (H * H) * GAN_HIDDEN + GAN_HIDDEN * 2 * H * H + 2 * GAN_HIDDEN
    return dict(gat=gat, time_encoder=te, encoder_layers=layers, decoders=dec, gan=gan)


def flops_per_window(H: int) -> dict:
    return {k: 2 * v for k, v in macs_per_window(H).items()}


def total_flops_per_window(H: int) -> int:
    return sum(flops_per_window(H).values())


def encdec_flops_per_window(H: int) -> int:
    """K2 (encdec_kernel): time encoder + 2 encoder layers + both decoders."""
    f = flops_per_window(H)
    return f["time_encoder"] + f["encoder_layers"] + f["decoders"]


def encoder_flops_per_window(H: int) -> int:
    """K2 (encoder_kernel): time encoder + 2 encoder layers."""
    f = flops_per_window(H)
    return f["time_encoder"] + f["encoder_layers"]


# MFMA instructions (v_mfma_f32_16x16x4_f32, 2,048 flops each, 16 windows) per
# host and wave in the encoder kernel's ISA (tools/isa_count.py).  K2 executes
# fewer MFMA flops than the reference's algorithm (layer-0 folds), so
# its algorithmic rate can exceed the peak; the executed rate cannot.
ENC_MFMA_PER_HOST = {16: 264, 50: 1116}


def encoder_executed_flops_per_window(H: int):
    n = ENC_MFMA_PER_HOST.get(H)
    return None if n is None else n * 2048 * H / 16


# The split feed-forward form (pgp_encoder.hip EncS, encoder_kernel<H, true>):
# (v_mfma_f32_16x16x4_f32, v_mfma_f32_16x16x32_bf16) per host and wave, ISA
# counted likewise (tools/isa_count.py encoder_split_counts).
ENC_SPLIT_MFMA_PER_HOST = {50: (516, 504)}


def encoder_split(H: int) -> bool:
    """K2 runs the split-bf16 feed-forward at these H (the tail-resident mode)."""
    return H in ENC_SPLIT_MFMA_PER_HOST


def encoder_split_executed_flops_per_window(H: int):
    """(fp32 MFMA flops, bf16 MFMA flops) K2's split form executes per window."""
    f32, bf = ENC_SPLIT_MFMA_PER_HOST[H]
    return f32 * 2048 * H / 16, bf * 16 * 16 * 32 * 2 * H / 16


# Fused tuning encoder (pgp_tunef.hip): v_mfma_f32_16x16x4_f32 per unit of 16
# (window, host) pairs, the static counts of the built ISA (tools/isa_count.py
# tune_counts, held equal by tests/test_roofline_isa.py).  tf_fwd_kernel's count
# includes layer 0's time encoder (tune_te_mfma), which layer 1 skips.  At H = 50
# the feed-forward GEMMs and out_proj's transpose run split-bf16
# (TF<H>::SPLIT): their v_mfma_f32_16x16x32_bf16 per unit in TUNE_BF16_PER_UNIT.
TUNE_MFMA_PER_UNIT = {
    16: {"tf_fwd_kernel": 156, "tf_bwd_ffn_kernel": 288, "tf_bwd_att_kernel": 96},
    50: {"tf_fwd_kernel": 840, "tf_bwd_ffn_kernel": 384, "tf_bwd_att_kernel": 1200},
}
TUNE_BF16_PER_UNIT = {
    16: {"tf_fwd_kernel": 0, "tf_bwd_ffn_kernel": 0, "tf_bwd_att_kernel": 0},
    50: {"tf_fwd_kernel": 288, "tf_bwd_ffn_kernel": 576, "tf_bwd_att_kernel": 144},
}
TUNE_FUSED_LAUNCHES = ("fwd layer 0", "fwd layer 1", "ffn bwd layer 1", "att bwd layer 1", "ffn bwd layer 0",
                       "att bwd layer 0")


def tf_grid(units: int, waves: int, cus: int, reserve: int = 0) -> int:
    """Workgroups of one fused tuning launch (mirrors pgp_tunef.hip
    tf_grid_for): the fewest workgroups whose longest wave has as many units
    as on the whole budget (cus - reserve, reserve capped at cus / 2)."""
    r = max(0, min(reserve, cus // 2))
    gmax = max(1, min(cus - r, (units + waves - 1) // waves))
    m = (units + waves * gmax - 1) // (waves * gmax)
    return max(1, (units + waves * m - 1) // (waves * m))


def tune_fused_grids(H: int, B: int, B_fwd: int | None, cus: int, reserve: int = 0):
    """Workgroups (= CUs held, one per CU) of the six fused launches, in
    TUNE_FUSED_LAUNCHES order: the forward's 8-wave workgroups over the
    forward batch's units, the backward's 4-wave ones over the backward's."""
    units = (B * H + 15) // 16
    ufwd = ((B if B_fwd is None else B_fwd) * H + 15) // 16
    gf, gb = tf_grid(ufwd, 8, cus, reserve), tf_grid(units, 4, cus, reserve)
    return [gf, gf, gb, gb, gb, gb]


def tune_te_mfma(H: int) -> int:
    """Time-encoder MFMAs per unit: NT output tiles x KS k-steps x 3 window steps."""
    nt = (H + 15) // 16
    ks = 4 * (H // 16) + (min(H % 16, 4) if H % 16 else 0)
    return nt * ks * 3


def tune_fused_flops(H: int, B: int, B_fwd: int | None = None):
    """Executed MFMA flops of each of the six fused launches of one tuning
    forward + backward (TUNE_FUSED_LAUNCHES order) over the batch's units; the
    FFN backward's zero rounds of waves past their units are not counted.
    B_fwd (default B): the forward's batch when it also carries inference
    windows (C3's detect) that the backward does not."""
    c = TUNE_MFMA_PER_UNIT.get(H)
    if c is None:
        return None
    # fp32-MFMA-equivalent work: a bf16 16x16x32 (16,384 flops) counted at the
    # fp32 / bf16 dense-peak ratio (1/16), so achieved / the fp32 peak is the
    # matrix pipe's busy fraction the executed work implies
    bf = TUNE_BF16_PER_UNIT.get(H, {})
    eq = {k: n * 2048 + bf.get(k, 0) * 16 * 16 * 32 * 2 * PEAK_FP32_TFLOPS / PEAK_BF16_TFLOPS for k, n in c.items()}
    units = (B * H + 15) // 16
    ufwd = ((B if B_fwd is None else B_fwd) * H + 15) // 16
    fwd, te = eq["tf_fwd_kernel"], tune_te_mfma(H) * 2048
    return ([ufwd * fwd, ufwd * (fwd - te)]
            + [units * n for n in (eq["tf_bwd_ffn_kernel"], eq["tf_bwd_att_kernel"], eq["tf_bwd_ffn_kernel"],
                                   eq["tf_bwd_att_kernel"])])


def encoder_io_bytes_per_window(H: int) -> int:
    """K2's own compulsory HBM I/O: the GAT output it reads (W x H x 3 aggregated
    raw features, fp32) and the latent it writes (3H^2 fp32) for K2b."""
    return 4 * (W * H * 3) + 4 * (W * H * H)


def decoder_flops_per_window(H: int) -> int:
    """K2b (decoder_kernel): anomaly + prototype decoders."""
    return flops_per_window(H)["decoders"]


def decoder_split(H: int) -> bool:
    """K2b runs the split-bf16 form at these H (pgp_decoder.hip dec_split: the
    LDS ring of one (host, step) chunk's three weight planes fits)."""
    return H in (32, 50)


def gan_split(H: int) -> bool:
    """K3 runs the split-bf16 form (pgp_gansplit.hip) at these H (batches of
    64 K windows and more)."""
    return H in (16, 50)


def gan_split_flops_per_window(H: int, onehot: bool = True) -> int:
    """bf16 MFMA flops K3's split form (pgp_gansplit.hip) executes per window:
    v_mfma_f32_16x16x32_bf16 (16 x 16 x 32 x 2 flops for 16 windows) counted
    per phase: Gen1 embedding pairs x 4 hidden tiles x 6; the schedule pass,
    pairs of 16-column blocks x 8 tiles (Gen1 | Disc1) x 3 (one-hot rows are
    exact in bf16) or 6; per container Gen2 (4 output tiles x 2 hidden pairs)
    and Disc1's new half (4 tiles x its pairs), 6 each."""
    ep = (2 * H + 15) // 16
    npe = (ep + 1) // 2
    nps = ((H * H + 15) // 16 + 1) // 2
    mtn = (H + 15) // 16
    npn = (mtn + 1) // 2
    n = npe * 4 * 6 + nps * 8 * (3 if onehot else 6) + H * (mtn * 2 * 6 + 4 * npn * 6)
    return n * 16 * 16 * 32 * 2 // 16


def decoder_split_flops_per_window(H: int) -> int:
    """bf16 MFMA flops K2b's split form executes per window: per (host, step)
    chunk ceil(KS/8) blocks of 8 k-steps (KS = ceil(H/4) k-steps of 4), per
    16-row output tile (ceil(4H/16)) 6 v_mfma_f32_16x16x32_bf16 of
    16 x 16 x 32 x 2 flops, shared by the 16 windows of a wave."""
    ks = (H + 3) // 4
    nb = ((ks + 3) // 4 + 1) // 2
    mt = (4 * H + 15) // 16
    return H * W * nb * mt * 6 * 16 * 16 * 32 * 2 // 16


def gan_flops_per_window(H: int) -> int:
    return flops_per_window(H)["gan"]


def path_bytes_per_window(H: int) -> int:
    """in 36H (window) + 4H^2 (dense schedule); out logits 8H,
    protos 8H, class 4H, final target 4H, probs 8."""
    return 36 * H + 4 * H * H + 8 * H + 8 * H + 4 * H + 4 * H + 8


def fpe_macs_per_window(H: int = 16) -> int:
    """PreGAN FPE_16 (models.py:65-115) on the reference's formulation: GRU,
    GAT (fc, decomposed scores, aggregation), MHA(E = H+3, 1 head), encoder,
    per-host decoders."""
    E, L = H + 3, 10
    gru = W * (9 * 3 * H + 9 * 3)
    gat = W * (H * 3 * H + 2 * H * H + H * H * H)
    mha = W * 3 * E * E + 2 * W * W * E + W * E * E
    enc = W * E * L * H
    dec = H * (2 * L + 2 * L)
    return gru + gat + mha + enc + dec


def fpe_flops_per_window(H: int = 16) -> int:
    return 2 * fpe_macs_per_window(H)


def fpe_executed_flops_per_window(H: int = 16) -> int:
    """Flops K4 (pgp_fpe.hip) executes per window, an FMA counted as 2 (a
    v_pk_fma_f32 as 4): per step the GRU input product (27 FMAs per node) and
    the node scores s, t (6), the GRU cell's hidden product (27), then per
    edge (i, j) one v_fma_f32 with output clamp (the branch indicator) and one
    v_pk_fma_f32 into {SA, SC}, per source node s_i (3 FMAs), its weight r_i
    and the r-weighted features (3); after the steps the 6x6 score form over
    3x3 token pairs and the [4H x 18] map.  Exponentials, compares and
    stores are not counted.  The reference's formulation (fpe_flops_per_window:
    H^3 GAT aggregation, E = H+3 MHA, 3E -> 10H encoder) is far larger; the
    kernel's algebra (rank-3 node mean, per-branch factorised edge softmax)
    removes that work, so the executed figure is the one priced against the
    VALU peak."""
    per_step = H * (27 + 6) * 2 + 27 * 2 + H * H * (2 + 4) + H * (3 + 3 + 2) * 2
    mha = 3 * (36 + 6) * 2 + 9 * 6 * 2 + 3 * 3 * 6 * 2
    out = 4 * H * 18 * 2
    return 3 * per_step + mha + out


def fpe_bytes_per_window(H: int = 16) -> int:
    """K4's compulsory HBM I/O: window 36H + h0 12 in; scores 8H, protos 8H,
    class 4H, any 4, masked embedding 8H (to K3) out."""
    return 36 * H + 12 + 8 * H + 8 * H + 4 * H + 4 + 8 * H


def tune_step_flops_per_window(H: int) -> int:
    """One window of the tuning step (train.py:42-57): the Transformer's forward
    (GAT, time encoder, 2 encoder layers, both decoders) and its backward, which
    for every dense product forms the input gradient and the weight gradient
    (2 x the forward's MACs): 3 x the forward's flops (the GAN is not trained
    by tune_model)."""
    f = flops_per_window(H)
    return 3 * (f["gat"] + f["time_encoder"] + f["encoder_layers"] + f["decoders"])


def gan_step_macs_per_env(H: int, hidden: int = GAN_HIDDEN) -> int:
    """One environment of train_gan (PreGANPlus.py:60-75) on the reference's
    formulation: Gen forward (Gen1 over [e; s], Gen2), Disc forward on [s; ns]
    (Disc1, head); Disc step: head and Disc1 weight gradients; Gen step: the
    updated Disc's forward again, d ns = Disc1[:, ns]^T dDD, Gen2's weight
    gradient, dHg = Gen2^T dY, Gen1's weight gradient."""
    gin, hh = 2 * H + H * H, H * H
    fwd = hidden * gin + hh * hidden + hidden * 2 * hh + 2 * hidden
    disc_step = 2 * hidden + 2 * hidden + hidden * 2 * hh            # head dW, dDD, Disc1 dW
    gen_step = hidden * 2 * hh + 2 * hidden + 2 * hidden + 3 * hh * hidden + hidden * gin
    return fwd + disc_step + gen_step


def gan_step_flops_per_env(H: int) -> int:
    return 2 * gan_step_macs_per_env(H)
