"""CPU restatement of PreGAN+'s decision model — TEST INFRASTRUCTURE ONLY.

This module is the parity oracle.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker
(or, in bench.py, as the timed CPU baseline).  The product path
(``preganplus_amd``) never imports it and fails loudly without its HIP library.

Plain numpy, batched over windows, H-generic, fp64 by default (the reference
runs fp64: ``recovery/PreGANSrc/src/utils.py:64``, ``recovery/PreGANPlus.py:117``)
with an optional fp32 mode.  Every function cites the reference code it restates
(paths relative to the reference repo root).  Semantics are those of the
reference modules in ``eval()`` mode (dropout off), which is how parity is
defined.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against
fixtures produced by importing the reference itself (``tests/golden/make_golden.py``)
on the shipped H=16 checkpoints and on seeded H=50 weights.  DGL (``dgl==0.7.2``,
reference ``README.md:42``) is absent from the image; its graph-wise
``softmax_edges`` is restated from DGL's published semantics (SURVEY.md §0.3,
§8c), so the GAT edge-softmax semantics are pinned only through that
restatement.
"""
from __future__ import annotations

import numpy as np

# recovery/PreGANSrc/src/constants.py:11-16
PERCENTILES = 98
PROTO_DIM = 2
PROTO_UPDATE_FACTOR = 0.2
PROTO_UPDATE_MIN = 0.02
PROTO_FACTOR_DECAY = 0.995
LATEST_WINDOW_SIZE = 10
# recovery/PreGANSrc/src/constants.py:19-20
COEFF_ENERGY = 0.8
COEFF_LATENCY = 0.2

N_WINDOW = 3      # models.py:320
N_FEATS = 3       # models.py:321 (cpu, ram, disk per host; stats/Stats.py:46-48)
N_HEADS = 2       # models.py:324
FF_DIM = 64       # models.py:325
N_LAYERS = 2      # models.py:326
GEN_HIDDEN = 64   # models.py:124 / :264
DISC_HIDDEN = 64  # models.py:142 / :282
LN_EPS = 1e-5     # torch.nn.TransformerEncoderLayer default layer_norm_eps


# ----------------------------------------------------------------------------
# pre-processing (recovery/PreGANSrc/src/utils.py)
# ----------------------------------------------------------------------------
def normalize_test_time_data(time_data, train_time_data):
    """utils.py:94-95: x / (colmax(train) + 1e-8)."""
    return time_data / (np.max(train_time_data, axis=0) + 1e-8)


def convert_to_windows(data, n_window=N_WINDOW):
    """utils.py:7-14: window i = rows [i-w, i) (row 0 repeated for i < w)."""
    data = np.asarray(data, dtype=np.float64)
    out = []
    for i in range(data.shape[0]):
        if i >= n_window:
            w = data[i - n_window:i]
        else:
            w = np.concatenate([np.repeat(data[0:1], n_window - i, axis=0), data[0:i]])
        out.append(w)
    return np.stack(out)


def inference_window(time_series, train_time_data, n_window=N_WINDOW):
    """PreGANPlus.py:107-112 (run_encoder's input selection).

    Normalise, keep the last ``n_window`` rows, ``convert_to_windows(...)[-1]``.
    The window used is rows [t-2, t-2, t-1]: the newest row is never seen.
    """
    t = normalize_test_time_data(np.asarray(time_series, dtype=np.float64),
                                 train_time_data)
    if t.shape[0] >= n_window:
        t = t[-n_window:]
    return convert_to_windows(t, n_window)[-1]


def form_test_dataset(data):
    """utils.py:16-24: per-host anomaly label (any of 3 columns above its 98th
    percentile over the rows) and class (argmax of the host's 3 columns)."""
    anomaly_per_dim = data > np.percentile(data, PERCENTILES, axis=0)
    which, anydim = [], []
    for i in range(0, data.shape[1], 3):
        which.append(np.argmax(data[:, i:i + 3] + 0, axis=1))
        anydim.append(np.logical_or.reduce(anomaly_per_dim[:, i:i + 3], axis=1))
    return np.stack(anydim, axis=1) + 0, np.stack(which, axis=1)


# ----------------------------------------------------------------------------
# model pieces
# ----------------------------------------------------------------------------
def _lin(x, w, b=None):
    # one 2-D GEMM over all leading axes (a stacked matmul calls BLAS per slice)
    y = (x.reshape(-1, x.shape[-1]) @ w.T).reshape(x.shape[:-1] + (w.shape[0],))
    if b is not None:
        y = y + b
    return y


def gat(win, fc_w, attn_w):
    """GAT layer: ``dlutils.py:304-348`` (GATHead) + ``:351-369`` (1-head mean).

    win: [B, W, H, 3] -> [B, W, H, d].  Fully connected graph, edges src-major
    (``models.py:332-334``: edge e = i*H + j, src i, dst j).
      z = fc(x)                                    (dlutils.py:315, no bias)
      e_ij = leaky_relu_0.01(a . [z_i || z_j])     (dlutils.py:326-329)
      a = softmax over ALL H*H edges per window step (dgl.softmax_edges, :335)
      h_j = sum_i a_ij z_i                         (update_all, :338-342)
    """
    z = win @ fc_w.T                                   # [B,W,H,d]
    d = fc_w.shape[0]
    a_src, a_dst = attn_w[0, :d], attn_w[0, d:]
    s = z @ a_src                                      # [B,W,H]  (src term)
    t = z @ a_dst                                      # [B,W,H]  (dst term)
    e = s[..., :, None] + t[..., None, :]              # [B,W,Hsrc,Hdst]
    e = np.where(e > 0, e, 0.01 * e)
    B, W, H = s.shape
    ef = e.reshape(B, W, H * H)
    ef = ef - ef.max(axis=-1, keepdims=True)
    p = np.exp(ef)
    p = (p / p.sum(axis=-1, keepdims=True)).reshape(B, W, H, H)
    return np.matmul(p.transpose(0, 1, 3, 2), z)       # sum_i p_ij z_i (einsum bwij,bwid->bwjd)


def layer_norm(x, g, b, eps=LN_EPS):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * g + b


def encoder_layer(x, p, n_heads=N_HEADS):
    """torch.nn.TransformerEncoderLayer(d, 2, 64, 0.1), post-norm, ReLU,
    batch_first=False, eval mode (``models.py:350-356``).

    x: [B, S=W, N=H, d].  Self-attention runs along the window axis S for each
    host N independently.
    """
    d = x.shape[-1]
    hd = d // n_heads
    qkv = _lin(x, p["in_proj_weight"], p["in_proj_bias"])       # [B,S,N,3d]
    q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
    B, S, N, _ = x.shape
    q = q.reshape(B, S, N, n_heads, hd)
    k = k.reshape(B, S, N, n_heads, hd)
    v = v.reshape(B, S, N, n_heads, hd)
    sc = np.einsum("bsnhe,btnhe->bnhst", q, k) / np.sqrt(hd)
    sc = sc - sc.max(-1, keepdims=True)
    pr = np.exp(sc)
    pr = pr / pr.sum(-1, keepdims=True)
    o = np.einsum("bnhst,btnhe->bsnhe", pr, v).reshape(B, S, N, d)
    sa = _lin(o, p["out_proj_weight"], p["out_proj_bias"])
    x = layer_norm(x + sa, p["norm1_weight"], p["norm1_bias"])
    ff = _lin(np.maximum(_lin(x, p["linear1_weight"], p["linear1_bias"]), 0.0),
              p["linear2_weight"], p["linear2_bias"])
    return layer_norm(x + ff, p["norm2_weight"], p["norm2_bias"])


def layer_params(tw, li):
    pre = f"transformer_encoder.layers.{li}."
    keys = ["self_attn.in_proj_weight", "self_attn.in_proj_bias",
            "self_attn.out_proj.weight", "self_attn.out_proj.bias",
            "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias",
            "norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias"]
    out = {}
    for k in keys:
        out[k.replace("self_attn.", "").replace(".", "_")] = tw[pre + k]
    return out


def encode(tw, win_flat, dtype=np.float64, return_gat=False):
    """``Transformer_16.encode`` (``models.py:376-400``), batched and H-generic.

    win_flat: [B, W, 3H] normalised windows -> latent [B, 3H^2] in the
    reference's (host, step, channel) order (``permute(1,0,2)``, :399).
    """
    tw = {k: np.asarray(v, dtype=dtype) for k, v in tw.items()}
    win_flat = np.asarray(win_flat, dtype=dtype)
    B, W, F = win_flat.shape
    H = F // N_FEATS
    x = win_flat.reshape(B, W, H, N_FEATS)
    g = gat(x, tw["gat.layer1.heads.0.fc.weight"], tw["gat.layer1.heads.0.attn_fc.weight"])
    h = _lin(g, tw["time_encoder.weight"], tw["time_encoder.bias"])      # :390
    h = h + tw["pos_encoder.pe"][:W].reshape(1, W, 1, -1)                # :309-311
    for li in range(N_LAYERS):
        h = encoder_layer(h, layer_params(tw, li))
    lat = np.transpose(h, (0, 2, 1, 3)).reshape(B, -1)                  # :399
    if return_gat:
        return lat, g
    return lat


def decode(tw, latent, dtype=np.float64):
    """``anomaly_decoder`` / ``prototype_decoder`` (``models.py:359-370``) and
    the per-host split (``:402-416``).  ``nn.LeakyReLU(True)`` has slope 1.0,
    i.e. it is the identity, so logits are raw linear outputs.
    Returns logits [B,H,2], protos [B,H,2]."""
    tw = {k: np.asarray(v, dtype=dtype) for k, v in tw.items()}
    B = latent.shape[0]
    a = _lin(latent, tw["anomaly_decoder.0.weight"], tw["anomaly_decoder.0.bias"])
    p = _lin(latent, tw["prototype_decoder.0.weight"], tw["prototype_decoder.0.bias"])
    p = 1.0 / (1.0 + np.exp(-p))
    return a.reshape(B, -1, 2), p.reshape(B, -1, PROTO_DIM)


def classify(logits, protos, prototypes):
    """Detect + embed (``PreGANPlus.py:119-131``) and ``get_classes``
    (``utils.py:102-109``).

    anomalous_h = first-argmax(logits_h) == 1  <=>  l1 > l0 (ties -> 0)
    emb_h       = proto_h if anomalous_h else 0
    class_h     = -1 if emb_h is all zero else first-argmin_k mean((emb_h-P_k)^2)
                  over the K = len(model.prototype) prototypes (16 for H=16).
    any_anom    = any_h anomalous_h   (else run_model returns the original decision)
    Returns anom [B,H] bool, emb [B,H,2], cls [B,H] int32, any [B] bool.
    """
    anom = logits[..., 1] > logits[..., 0]
    emb = np.where(anom[..., None], protos, 0.0)
    P = np.asarray(prototypes, dtype=emb.dtype)                        # [K,2]
    dist = ((emb[:, :, None, :] - P[None, None]) ** 2).mean(-1)        # [B,H,K]
    cls = np.argmin(dist, axis=-1).astype(np.int32)
    zero = np.all(emb == 0, axis=-1)
    cls = np.where(zero, -1, cls).astype(np.int32)
    return anom, emb, cls, anom.any(axis=1)


def class_margin(emb, prototypes):
    """Top-2 gap of the class distances (0 where no class): used by the tests to
    tell a genuine near-tie from a kernel bug."""
    P = np.asarray(prototypes, dtype=np.float64)
    dist = ((emb[:, :, None, :].astype(np.float64) - P[None, None]) ** 2).mean(-1)
    srt = np.sort(dist, axis=-1)
    return srt[..., 1] - srt[..., 0]


def generator(gw, emb, sched, dtype=np.float64):
    """``Gen_16``/``Gen_50`` forward (``models.py:118-133, 258-273``):
    ns = s + 4*tanh(W2 . lrelu_1.0(W1 . [vec(emb), vec(s)] + b1) + b2)."""
    gw = {k: np.asarray(v, dtype=dtype) for k, v in gw.items()}
    B, C, H = sched.shape
    inp = np.concatenate([emb.reshape(B, -1), sched.reshape(B, -1)], axis=1).astype(dtype)
    h1 = _lin(inp, gw["delta.0.weight"], gw["delta.0.bias"])       # LeakyReLU(True) = id
    d = np.tanh(_lin(h1, gw["delta.2.weight"], gw["delta.2.bias"]))
    return sched + 4.0 * d.reshape(B, C, H)


def discriminator(dw, sched, new_sched, dtype=np.float64):
    """``Disc_16``/``Disc_50`` forward (``models.py:136-151, 276-291``):
    probs = softmax(W2 . lrelu_1.0(W1 . [vec(s), vec(ns)] + b1) + b2)."""
    dw = {k: np.asarray(v, dtype=dtype) for k, v in dw.items()}
    B = sched.shape[0]
    inp = np.concatenate([sched.reshape(B, -1), new_sched.reshape(B, -1)], axis=1).astype(dtype)
    h1 = _lin(inp, dw["probs.0.weight"], dw["probs.0.bias"])
    z = _lin(h1, dw["probs.2.weight"], dw["probs.2.bias"])
    z = z - z.max(-1, keepdims=True)
    e = np.exp(z)
    return e / e.sum(-1, keepdims=True)


def first_argmax_rows(m):
    """``list.index(max(list))`` per row (``PreGANPlus.py:98-99``,
    ``stats/Stats.py:163-165``): the first maximal index."""
    return np.argmax(m, axis=-1).astype(np.int32)


def decide(sched, new_sched, probs):
    """Decision tensors of ``recover_decision`` (``PreGANPlus.py:84-105``):
    keep_orig = p0 > p1 (strict, :87); final_target = first-argmax of the
    ORIGINAL schedule rows (:99); gen_target = first-argmax of the generator's
    rows (the proposal scored by ``Stats.runSimulation``, Stats.py:162-166)."""
    keep = probs[:, 0] > probs[:, 1]
    return keep, first_argmax_rows(sched), first_argmax_rows(new_sched)


def forward(weights, windows, sched, dtype=np.float64):
    """detect + diagnose + generate for a batch of windows.

    weights: dict with 'transformer', 'gen', 'disc' state dicts (numpy) and
    'prototypes' [K,2].  windows [B,W,3H] (normalised), sched [B,C,H].
    """
    lat = encode(weights["transformer"], windows, dtype)
    logits, protos = decode(weights["transformer"], lat, dtype)
    anom, emb, cls, anyb = classify(logits, protos, weights["prototypes"])
    sched = np.asarray(sched, dtype=dtype)
    ns = generator(weights["gen"], emb, sched, dtype)
    probs = discriminator(weights["disc"], sched, ns, dtype)
    keep, final_t, gen_t = decide(sched, ns, probs)
    return dict(latent=lat, logits=logits, protos=protos, anom=anom, emb=emb,
                cls=cls, any=anyb, new_sched=ns, probs=probs, keep=keep,
                final_target=final_t, gen_target=gen_t)


def recover_decision_list(keep, sched_row_targets, containers, n_hosts, original_decision):
    """Decision assembly of ``recover_decision`` (``PreGANPlus.py:87-105``).

    containers: list of (cid, host_id) for placed containers in containerlist
    order (host -1 / None excluded by the caller).  Returns (decision list,
    hosts_from)."""
    if keep:
        return list(original_decision), None
    host_alloc = [[] for _ in range(n_hosts)]
    container_alloc = {}
    for cid, hid in containers:
        host_alloc[hid].append(cid)
        container_alloc[cid] = hid
    decision = dict(original_decision)
    hosts_from = [0] * n_hosts
    for hid in range(n_hosts):
        for cid in host_alloc[hid]:
            new_host = int(sched_row_targets[cid])
            if container_alloc[cid] != new_host:
                decision[cid] = new_host
                hosts_from[container_alloc[cid]] = 1
    return list(decision.items()), hosts_from


def positional_encoding(d_model, max_len=N_WINDOW):
    """``PositionalEncoding`` buffer (``models.py:297-307``), computed in fp32 as
    the reference does before ``.double()``; shape [max_len, 1, d]."""
    position = np.arange(0, max_len, dtype=np.float32)[:, None]
    div = np.exp(np.arange(0, d_model, 2, dtype=np.float32)
                 * np.float32(-np.log(10000.0) / d_model)).astype(np.float32)
    pe = np.zeros((max_len, d_model), dtype=np.float32)
    pe[:, 0::2] = np.sin(position * div)
    pe[:, 1::2] = np.cos(position * div)
    return pe.astype(np.float64)[:, None, :]


# ----------------------------------------------------------------------------
# PreGAN's FPE_16 encoder (models.py:10-115) — BASELINE config 4
# ----------------------------------------------------------------------------
def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def fpe_forward(fw, win_flat, h0, dtype=np.float64):
    """``FPE_16.forward`` (models.py:65-115), batched.

    win_flat [B,3,3H] normalised windows; h0 [B,3] GRU initial state (the
    reference draws it with torch.randn inside encode, models.py:70, so it is an
    explicit input here).  Returns per-host anomaly softmax probs [B,H,2] and
    sigmoid prototypes [B,H,2].
      GRU(3H -> 3) over the 3 window rows (torch gate order r, z, n)
      GAT over [1,3,H,3] (dlutils.py:304-348), mean over nodes -> [3, H]
      concat -> [3,1,3+H] -> MultiheadAttention(3+H, 1 head), seq 3, batch 1
      flatten [3*(3+H)] -> Linear -> H x 10 latent (LeakyReLU(True) = id)
      per host: Softmax(Linear(10,2)) and Sigmoid(Linear(10,2)).
    """
    fw = {k: np.asarray(v, dtype=dtype) for k, v in fw.items()}
    x = np.asarray(win_flat, dtype=dtype)
    B, Wn, F = x.shape
    H = F // 3
    h = np.asarray(h0, dtype=dtype).reshape(B, 3)
    Wih, Whh, bih, bhh = fw["gru.weight_ih_l0"], fw["gru.weight_hh_l0"], fw["gru.bias_ih_l0"], fw["gru.bias_hh_l0"]
    gru = []
    for w in range(Wn):
        gi = x[:, w] @ Wih.T + bih
        gh = h @ Whh.T + bhh
        r = _sigmoid(gi[:, 0:3] + gh[:, 0:3])
        z = _sigmoid(gi[:, 3:6] + gh[:, 3:6])
        n = np.tanh(gi[:, 6:9] + r * gh[:, 6:9])
        h = (1 - z) * n + z * h
        gru.append(h)
    gru = np.stack(gru, axis=1)                                                   # [B,3,3]
    g = gat(x.reshape(B, Wn, H, 3), fw["gat.layer1.heads.0.fc.weight"],
            fw["gat.layer1.heads.0.attn_fc.weight"]).mean(axis=2)                 # [B,3,H]
    c = np.concatenate([gru, g], axis=2)                                          # [B,3,E]
    E = c.shape[2]
    qkv = c @ fw["mha.in_proj_weight"].T + fw["mha.in_proj_bias"]
    q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    sc = np.einsum("bse,bte->bst", q, k) / np.sqrt(E)
    sc = sc - sc.max(-1, keepdims=True)
    p = np.exp(sc)
    p = p / p.sum(-1, keepdims=True)
    o = np.einsum("bst,bte->bse", p, v) @ fw["mha.out_proj.weight"].T + fw["mha.out_proj.bias"]
    lat = (o.reshape(B, -1) @ fw["encoder.0.weight"].T + fw["encoder.0.bias"]).reshape(B, H, -1)
    a = lat @ fw["anomaly_decoder.0.weight"].T + fw["anomaly_decoder.0.bias"]
    a = a - a.max(-1, keepdims=True)
    a = np.exp(a)
    probs = a / a.sum(-1, keepdims=True)
    protos = _sigmoid(lat @ fw["prototype_decoder.0.weight"].T + fw["prototype_decoder.0.bias"])
    return probs, protos


def forward_fpe(weights, windows, h0, sched, dtype=np.float64):
    """PreGAN (``recovery/PreGAN.py:97-126``) per-window path: FPE encoder,
    detect (argmax of the softmax == 1), embed, classes over K=3 prototypes,
    Gen/Disc and the decision tensors."""
    probs, protos = fpe_forward(weights["fpe"], windows, h0, dtype)
    anom, emb, cls, anyb = classify(probs, protos, weights["prototypes"])
    sched = np.asarray(sched, dtype=dtype)
    ns = generator(weights["gen"], emb, sched, dtype)
    gp = discriminator(weights["disc"], sched, ns, dtype)
    keep, final_t, gen_t = decide(sched, ns, gp)
    return dict(probs=probs, protos=protos, anom=anom, emb=emb, cls=cls, any=anyb, new_sched=ns,
                gprobs=gp, keep=keep, final_target=final_t, gen_target=gen_t)
