"""CPU restatement of PreGAN+'s online training steps — TEST INFRASTRUCTURE ONLY.

Same status as ``pregan_oracle``: imported only by tests/, smoke() and bench.py's
CPU baseline, never by the product.  It restates, with torch autograd on the CPU
(fp64 by default; a floating-point reference, as allowed for fp kernels):

* the semi-supervised tuning step: ``backprop`` (train.py:42-57),
  ``custom_loss`` (train.py:27-40), ``triplet_loss`` (train.py:13-25), the
  on-the-fly dataset (utils.py:16-24, 40-47), and AdamW as torch implements it
  (utils.py:65: lr = model.lr, weight_decay 1e-5, betas (0.9, 0.999), eps 1e-8);
* the online GAN step ``train_gan`` (PreGANPlus.py:60-81) with BCELoss;
* ``run_model`` (PreGANPlus.py:115-136) on a duck-typed environment.

Dropout is 0 (the reference never calls eval(); parity is defined with dropout
off).  The reference keeps PROTO_UPDATE_FACTOR / num_zero /
num_ones as module globals (train.py:1-11); here they live in ``TuneState``.
Pinned by tests/test_train_oracle_golden.py against fixtures produced by the
reference itself (tests/golden/make_golden_train.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import pregan_oracle as O

T = torch


# ---------------------------------------------------------------------------
# model forward in torch (same math as pregan_oracle.encode/decode, batched)
# ---------------------------------------------------------------------------
def _lin(x, w, b=None):
    y = x @ w.T
    return y + b if b is not None else y


def encode_t(tw, win):
    """win [B,W,3H] -> latent [B,3H^2] (models.py:376-400)."""
    B, Wn, F = win.shape
    H = F // 3
    x = win.reshape(B, Wn, H, 3)
    fc, at = tw["gat.layer1.heads.0.fc.weight"], tw["gat.layer1.heads.0.attn_fc.weight"]
    z = x @ fc.T
    d = fc.shape[0]
    s = z @ at[0, :d]
    t = z @ at[0, d:]
    e = s[..., :, None] + t[..., None, :]
    e = T.nn.functional.leaky_relu(e, 0.01)
    a = T.softmax(e.reshape(B, Wn, H * H), dim=-1).reshape(B, Wn, H, H)
    g = T.einsum("bwij,bwid->bwjd", a, z)
    h = _lin(g, tw["time_encoder.weight"], tw["time_encoder.bias"])
    h = h + tw["pos_encoder.pe"][:Wn].reshape(1, Wn, 1, -1)
    for li in range(2):
        p = f"transformer_encoder.layers.{li}."
        hd = d // 2
        qkv = _lin(h, tw[p + "self_attn.in_proj_weight"], tw[p + "self_attn.in_proj_bias"])
        q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
        q = q.reshape(B, Wn, H, 2, hd)
        k = k.reshape(B, Wn, H, 2, hd)
        v = v.reshape(B, Wn, H, 2, hd)
        sc = T.einsum("bsnhe,btnhe->bnhst", q, k) / math.sqrt(hd)
        pr = T.softmax(sc, dim=-1)
        o = T.einsum("bnhst,btnhe->bsnhe", pr, v).reshape(B, Wn, H, d)
        sa = _lin(o, tw[p + "self_attn.out_proj.weight"], tw[p + "self_attn.out_proj.bias"])
        h = T.nn.functional.layer_norm(h + sa, (d,), tw[p + "norm1.weight"], tw[p + "norm1.bias"], 1e-5)
        ff = _lin(T.relu(_lin(h, tw[p + "linear1.weight"], tw[p + "linear1.bias"])),
                  tw[p + "linear2.weight"], tw[p + "linear2.bias"])
        h = T.nn.functional.layer_norm(h + ff, (d,), tw[p + "norm2.weight"], tw[p + "norm2.bias"], 1e-5)
    return h.permute(0, 2, 1, 3).reshape(B, -1)


def decode_t(tw, lat):
    B = lat.shape[0]
    a = _lin(lat, tw["anomaly_decoder.0.weight"], tw["anomaly_decoder.0.bias"]).reshape(B, -1, 2)
    p = T.sigmoid(_lin(lat, tw["prototype_decoder.0.weight"], tw["prototype_decoder.0.bias"])).reshape(B, -1, 2)
    return a, p


def gen_t(gw, emb, s):
    B = s.shape[0]
    x = T.cat([emb.reshape(B, -1), s.reshape(B, -1)], 1)
    y = _lin(_lin(x, gw["delta.0.weight"], gw["delta.0.bias"]), gw["delta.2.weight"], gw["delta.2.bias"])
    return s + 4 * T.tanh(y).reshape(s.shape)


def disc_t(dw, s, ns):
    B = s.shape[0]
    x = T.cat([s.reshape(B, -1), ns.reshape(B, -1)], 1)
    z = _lin(_lin(x, dw["probs.0.weight"], dw["probs.0.bias"]), dw["probs.2.weight"], dw["probs.2.bias"])
    return T.softmax(z, dim=-1)


def fpe_t(fw, win, h0):
    """PreGAN's FPE_16 forward (models.py:65-115) in torch, batched: win [B,3,3H],
    h0 [B,3] (the GRU state models.py:70 draws) -> per-host anomaly softmax
    probabilities [B,H,2] and sigmoid prototypes [B,H,2].  Same math as
    pregan_oracle.fpe_forward (pinned to the reference's fixtures), with
    autograd: the offline-training restatement (PreGAN.py:39-49)."""
    B, Wn, F = win.shape
    H = F // 3
    h = h0.reshape(B, 3)
    Wih, Whh, bih, bhh = fw["gru.weight_ih_l0"], fw["gru.weight_hh_l0"], fw["gru.bias_ih_l0"], fw["gru.bias_hh_l0"]
    gru = []
    for w in range(Wn):
        gi = _lin(win[:, w], Wih, bih)
        gh = _lin(h, Whh, bhh)
        r = T.sigmoid(gi[:, 0:3] + gh[:, 0:3])
        z = T.sigmoid(gi[:, 3:6] + gh[:, 3:6])
        n = T.tanh(gi[:, 6:9] + r * gh[:, 6:9])
        h = (1 - z) * n + z * h
        gru.append(h)
    gru = T.stack(gru, 1)                                                         # [B,3,3]
    fc, at = fw["gat.layer1.heads.0.fc.weight"], fw["gat.layer1.heads.0.attn_fc.weight"]
    x = win.reshape(B, Wn, H, 3)
    z = x @ fc.T                                                                  # [B,W,H,d]
    d = fc.shape[0]
    e = T.nn.functional.leaky_relu((z @ at[0, :d])[..., :, None] + (z @ at[0, d:])[..., None, :], 0.01)
    a = T.softmax(e.reshape(B, Wn, H * H), dim=-1).reshape(B, Wn, H, H)       # graph-wise (all edges)
    g = T.einsum("bwij,bwid->bwjd", a, z).mean(dim=2)                            # node mean [B,W,d]
    c = T.cat([gru, g], 2)
    E = c.shape[2]
    qkv = _lin(c, fw["mha.in_proj_weight"], fw["mha.in_proj_bias"])
    q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
    p = T.softmax(T.einsum("bse,bte->bst", q, k) / math.sqrt(E), dim=-1)
    o = _lin(T.einsum("bst,bte->bse", p, v), fw["mha.out_proj.weight"], fw["mha.out_proj.bias"])
    lat = _lin(o.reshape(B, -1), fw["encoder.0.weight"], fw["encoder.0.bias"]).reshape(B, H, -1)
    probs = T.softmax(_lin(lat, fw["anomaly_decoder.0.weight"], fw["anomaly_decoder.0.bias"]), dim=-1)
    protos = T.sigmoid(_lin(lat, fw["prototype_decoder.0.weight"], fw["prototype_decoder.0.bias"]))
    return probs, protos


# ---------------------------------------------------------------------------
# AdamW exactly as torch.optim.AdamW (single-tensor path)
# ---------------------------------------------------------------------------
class AdamW:
    def __init__(self, params: dict, lr, state=None, wd=1e-5, betas=(0.9, 0.999), eps=1e-8):
        self.p = params                      # name -> leaf tensor
        self.lr, self.wd, self.b1, self.b2, self.eps = lr, wd, betas[0], betas[1], eps
        self.m, self.v, self.step = {}, {}, {}
        for n, q in params.items():
            st = (state or {}).get(n)
            self.m[n] = T.tensor(st["exp_avg"]) if st else T.zeros_like(q)
            self.v[n] = T.tensor(st["exp_avg_sq"]) if st else T.zeros_like(q)
            self.step[n] = float(st["step"]) if st else 0.0

    def zero_grad(self):
        for q in self.p.values():
            q.grad = None

    @T.no_grad()
    def apply(self):
        for n, q in self.p.items():
            if q.grad is None:
                continue
            g = q.grad
            self.step[n] += 1
            q.mul_(1 - self.lr * self.wd)
            self.m[n].lerp_(g, 1 - self.b1)
            self.v[n].mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
            bc1 = 1 - self.b1 ** self.step[n]
            bc2 = 1 - self.b2 ** self.step[n]
            denom = (self.v[n].sqrt() / math.sqrt(bc2)).add_(self.eps)
            q.addcdiv_(self.m[n], denom, value=-self.lr / bc1)


def opt_state_from_npz(extra: dict, prefix: str):
    st = {}
    for k, v in extra.items():
        if not k.startswith(f"opt/{prefix}/"):
            continue
        name, field = k[len(f"opt/{prefix}/"):].rsplit("/", 1)
        st.setdefault(name, {})[field] = v
    return st


def leaf_params(sd: dict, skip=("pos_encoder.pe",), dtype=T.float64):
    return {k: T.tensor(np.asarray(v), dtype=dtype, requires_grad=k not in skip) for k, v in sd.items()}


# ---------------------------------------------------------------------------
# tuning step
# ---------------------------------------------------------------------------
class TuneState:
    """Module globals of train.py (PROTO_UPDATE_FACTOR, num_zero, num_ones) and
    model.prototype (list of [2] tensors)."""

    def __init__(self, prototypes, factor=O.PROTO_UPDATE_FACTOR):
        self.protos = [T.tensor(np.asarray(p, dtype=np.float64)) for p in prototypes]
        self.factor = float(factor)
        self.num_zero, self.num_ones = 1, 1


def triplet_loss(anchor, c, st: TuneState):
    """train.py:13-25: positive MSE to the (detached) prototype minus the sum of
    the negatives' MSE values as a constant; EMA update of P[c] if the positive
    distance is the smallest of the three."""
    pos = T.mean((anchor - st.protos[c].detach().clone()) ** 2)
    negs = [nc for nc in (0, 1, 2) if nc != c]
    nl = [T.mean((anchor - st.protos[nc]) ** 2) for nc in negs]
    loss = pos - T.sum(T.tensor([float(x) for x in nl], dtype=anchor.dtype))
    if pos <= nl[0] and pos <= nl[1]:
        f = st.factor + O.PROTO_UPDATE_MIN
        st.protos[c] = (f * anchor + (1 - f) * st.protos[c]).detach()
    return loss


def custom_loss(logits, protos, y, c, st: TuneState):
    """train.py:27-40 for one window (logits [H,2], protos [H,2])."""
    nz, no = 0, 0
    aloss = 0
    tloss = T.tensor(0.0, dtype=logits.dtype)
    for i in range(logits.shape[0]):
        mult = 1 if y[i] == 0 else st.num_zero / st.num_ones
        nz += 1                      # (train.py:34 counts every host)
        no += 1 if y[i] == 1 else 0
        aloss = aloss + T.nn.functional.cross_entropy(logits[i:i + 1], T.tensor([int(y[i])])) * mult
    for i in range(protos.shape[0]):
        if y[i] > 0:
            tloss = tloss + triplet_loss(protos[i], int(c[i]), st)
    st.factor *= O.PROTO_FACTOR_DECAY
    st.num_zero += nz
    st.num_ones += no
    return aloss, tloss


def on_the_fly_dataset(time_series, schedule_series, train_time_data):
    """utils.py:40-47."""
    td = O.normalize_test_time_data(np.asarray(time_series)[-O.LATEST_WINDOW_SIZE:], train_time_data)
    sched = np.asarray(schedule_series)[-O.LATEST_WINDOW_SIZE:]
    wins = O.convert_to_windows(td)
    anom, cls = O.form_test_dataset(td)
    return wins, sched, anom, cls


def backprop(tw: dict, opt: AdamW, st: TuneState, wins, sched, anom, cls, record=None):
    """train.py:42-57: sequential batch-1 steps."""
    st.num_zero, st.num_ones = 1, 1
    losses = []
    for i in range(wins.shape[0]):
        lat = encode_t(tw, T.tensor(wins[i:i + 1]))
        logits, protos = decode_t(tw, lat)
        aloss, tloss = custom_loss(logits[0], protos[0], anom[i], cls[i], st)
        opt.zero_grad()
        (aloss + tloss).backward()
        if record is not None and i == 0:
            record["g0"] = {n: (q.grad.detach().numpy().copy() if q.grad is not None else None)
                            for n, q in tw.items()}
        opt.apply()
        if record is not None and i == 0:
            record["p1"] = {n: q.detach().numpy().copy() for n, q in tw.items()}
        losses.append((float(aloss), float(tloss)))
    return losses


def fpe_backprop(fw: dict, opt: AdamW, st: TuneState, wins, h0s, anom, cls):
    """train.py:42-57 for PreGAN's FPE_16 (PreGAN.py:39-49, train_model): the
    same sequential batch-1 loop and custom_loss as the Transformer's, on the
    FPE's outputs (its anomaly decoder ends in a Softmax, so CrossEntropyLoss
    sees probabilities, models.py:49-52); h0s [n,3]: the GRU state each
    forward drew.  Returns the per-window (aloss, tloss)."""
    st.num_zero, st.num_ones = 1, 1
    losses = []
    for i in range(wins.shape[0]):
        probs, protos = fpe_t(fw, T.tensor(wins[i:i + 1]), T.tensor(h0s[i:i + 1]))
        aloss, tloss = custom_loss(probs[0], protos[0], anom[i], cls[i], st)
        opt.zero_grad()
        (aloss + tloss).backward()
        opt.apply()
        losses.append((float(aloss), float(tloss)))
    return losses


# ---------------------------------------------------------------------------
# GAN step
# ---------------------------------------------------------------------------
def bce(p, target):
    """nn.BCELoss (mean; log clamped at -100)."""
    lp = T.clamp(T.log(p), min=-100)
    l1p = T.clamp(T.log(1 - p), min=-100)
    return -(target * lp + (1 - target) * l1p).mean()


def train_gan(gw, dw, gopt: AdamW, dopt: AdamW, emb, sched, simulate):
    """PreGANPlus.py:60-81.  ``simulate(schedule) -> score`` plays
    run_simulation (utils.py:97-100); returns (gen_loss, disc_loss, ns)."""
    emb = T.as_tensor(emb)
    s = T.as_tensor(sched)
    dopt.zero_grad()
    ns = gen_t(gw, emb[None], s[None])[0]
    probs = disc_t(dw, s[None], ns.detach()[None])[0]
    new_score, orig_score = simulate(ns.detach().numpy()), simulate(s.numpy())
    tp = T.tensor([0.0, 1.0] if new_score <= orig_score else [1.0, 0.0], dtype=probs.dtype)
    dloss = bce(probs, tp)
    dloss.backward()
    dopt.apply()
    gopt.zero_grad()
    dopt.zero_grad()
    probs = disc_t(dw, s[None], ns[None])[0]
    gloss = bce(probs, T.tensor([0.0, 1.0], dtype=probs.dtype))
    gloss.backward()
    gopt.apply()
    return float(gloss), float(dloss), ns.detach().numpy()


# ---------------------------------------------------------------------------
# run_model (PreGANPlus.py:115-136)
# ---------------------------------------------------------------------------
class PluginOracle:
    """Restatement of PreGANPlusRecovery's per-interval behaviour."""

    def __init__(self, weights: dict, extra: dict, train_time_data, factor=O.PROTO_UPDATE_FACTOR,
                 lrs=(1e-4, 5e-5, 5e-5)):
        self.tw = leaf_params(weights["transformer"])
        self.gw = leaf_params(weights["gen"], skip=())
        self.dw = leaf_params(weights["disc"], skip=())
        self.topt = AdamW({k: v for k, v in self.tw.items() if v.requires_grad}, lrs[0],
                          opt_state_from_npz(extra, "transformer"))
        self.gopt = AdamW(self.gw, lrs[1], opt_state_from_npz(extra, "gen"))
        self.dopt = AdamW(self.dw, lrs[2], opt_state_from_npz(extra, "disc"))
        self.st = TuneState(weights["prototypes"], factor)
        self.train_time = np.asarray(train_time_data, dtype=np.float64)

    def run_model(self, env, original_decision):
        s = T.tensor(np.asarray(env.scheduler.result_cache, dtype=np.float64))
        win = O.inference_window(env.stats.time_series, self.train_time)
        with T.no_grad():
            logits, protos = decode_t(self.tw, encode_t(self.tw, T.tensor(win[None])))
        logits, protos = logits[0], protos[0]
        anom = logits[:, 1] > logits[:, 0]
        if not bool(anom.any()):
            return list(original_decision)
        emb = T.where(anom[:, None], protos, T.zeros_like(protos))
        # train_gan
        scores = lambda sch: (lambda e, r: O.COEFF_ENERGY * e + O.COEFF_LATENCY * r)(
            *env.stats.runSimulation(T.tensor(sch)))
        train_gan(self.gw, self.dw, self.gopt, self.dopt, emb, s, scores)
        # tune_model
        wins, sched, an, cl = on_the_fly_dataset(env.stats.time_series, env.stats.schedule_series,
                                                 self.train_time)
        backprop(self.tw, self.topt, self.st, wins, sched, an, cl)
        # recover_decision
        with T.no_grad():
            ns = gen_t(self.gw, emb[None], s[None])
            probs = disc_t(self.dw, s[None], ns)[0]
        if probs[0] > probs[1]:
            return list(original_decision)
        containers = [(c.id, c.getHostID()) for c in env.containerlist if c and c.getHostID() != -1]
        targets = O.first_argmax_rows(s.numpy()[None])[0]
        dec, _ = O.recover_decision_list(False, targets, containers, len(env.hostlist), original_decision)
        return dec
