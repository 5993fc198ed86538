"""Weight sets for the PreGAN+ decision model (host side).

Two sources, both yielding the reference's own parameter names and shapes
(``recovery/PreGANSrc/src/models.py:314-416`` Transformer_16, ``:118-151``
Gen_16/Disc_16, ``:258-291`` Gen_50/Disc_50; checkpoint dict format
``recovery/PreGANSrc/src/utils.py:53-58``):

* :func:`load_reference_checkpoints` reads the shipped ``.ckpt`` files with
  ``torch.load(weights_only=True)`` (no code from the file runs);
* :func:`synth_weights` builds seeded random weights of the H-generic
  architecture (H=50 has no shipped checkpoint).  numpy's PCG64
  stream is platform-independent, so the same seed gives bit-identical weights
  on the build container and on the GPU box (the golden fixtures rely on it).

The packed blob handed to the C-ABI (``pgp_load_weights``) is the
concatenation, in :func:`blob_layout` order, of these arrays as float64.
"""
from __future__ import annotations

import os

import numpy as np

PROTO_DIM = 2


def transformer_shapes(H, W=3, ff=64, layers=2, feats=3):
    d = H
    shp = {
        "gat.layer1.heads.0.fc.weight": (d, feats),
        "gat.layer1.heads.0.attn_fc.weight": (1, 2 * d),
        "time_encoder.weight": (d, d),
        "time_encoder.bias": (d,),
        "pos_encoder.pe": (W, 1, d),
    }
    for li in range(layers):
        p = f"transformer_encoder.layers.{li}."
        shp.update({
            p + "self_attn.in_proj_weight": (3 * d, d),
            p + "self_attn.in_proj_bias": (3 * d,),
            p + "self_attn.out_proj.weight": (d, d),
            p + "self_attn.out_proj.bias": (d,),
            p + "linear1.weight": (ff, d),
            p + "linear1.bias": (ff,),
            p + "linear2.weight": (d, ff),
            p + "linear2.bias": (d,),
            p + "norm1.weight": (d,),
            p + "norm1.bias": (d,),
            p + "norm2.weight": (d,),
            p + "norm2.bias": (d,),
        })
    lat = H * d * W
    shp.update({
        "anomaly_decoder.0.weight": (2 * H, lat),
        "anomaly_decoder.0.bias": (2 * H,),
        "prototype_decoder.0.weight": (PROTO_DIM * H, lat),
        "prototype_decoder.0.bias": (PROTO_DIM * H,),
    })
    return shp


def gen_shapes(H, hidden=64):
    n = H * PROTO_DIM + H * H
    return {"delta.0.weight": (hidden, n), "delta.0.bias": (hidden,),
            "delta.2.weight": (H * H, hidden), "delta.2.bias": (H * H,)}


def disc_shapes(H, hidden=64):
    n = 2 * H * H
    return {"probs.0.weight": (hidden, n), "probs.0.bias": (hidden,),
            "probs.2.weight": (2, hidden), "probs.2.bias": (2,)}


def fpe_shapes(H=16, window=3, latent=10, feats=3):
    """PreGAN's ``FPE_16`` parameters in ``state_dict`` order (models.py:10-64)."""
    E = window + H                    # GRU state (3) + GAT node-mean (H)
    return {
        "gru.weight_ih_l0": (3 * window, feats * H), "gru.weight_hh_l0": (3 * window, window),
        "gru.bias_ih_l0": (3 * window,), "gru.bias_hh_l0": (3 * window,),
        "gat.layer1.heads.0.fc.weight": (H, feats), "gat.layer1.heads.0.attn_fc.weight": (1, 2 * H),
        "mha.in_proj_weight": (3 * E, E), "mha.in_proj_bias": (3 * E,),
        "mha.out_proj.weight": (E, E), "mha.out_proj.bias": (E,),
        "encoder.0.weight": (H * latent, window * E), "encoder.0.bias": (H * latent,),
        "anomaly_decoder.0.weight": (2, latent), "anomaly_decoder.0.bias": (2,),
        "prototype_decoder.0.weight": (PROTO_DIM, latent), "prototype_decoder.0.bias": (PROTO_DIM,),
    }


FPE_PROTOS = 3   # models.py:62


def fpe_blob_layout(H=16):
    """(section, name, shape) list of the PreGAN (FPE) variant's weight blob."""
    out = [("fpe", k, s) for k, s in fpe_shapes(H).items()]
    out += [("gen", k, s) for k, s in gen_shapes(H).items()]
    out += [("disc", k, s) for k, s in disc_shapes(H).items()]
    out += [("prototypes", "prototypes", (FPE_PROTOS, PROTO_DIM))]
    return out


def synth_fpe_weights(H=16, seed=0):
    """Seeded FPE + GAN weights (uniform +-1/sqrt(fan_in), fp32-representable)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    w = {}
    for sec, shapes in (("fpe", fpe_shapes(H)), ("gen", gen_shapes(H)), ("disc", disc_shapes(H))):
        w[sec] = {}
        for name, shp in shapes.items():
            if name.startswith("gru."):
                fan_in = 3
            elif len(shp) == 2:
                fan_in = shp[1]
            else:
                fan_in = shapes[name.replace("bias", "weight")][1]
            a = rng.uniform(-1, 1, size=shp) / np.sqrt(fan_in)
            w[sec][name] = a.astype(np.float32).astype(np.float64)
    w["prototypes"] = rng.uniform(0, 1, size=(FPE_PROTOS, PROTO_DIM)).astype(np.float32).astype(np.float64)
    return w


def blob_layout(H, n_protos=None):
    """Ordered (section, name, shape) list of the C-ABI weight blob."""
    K = H if n_protos is None else n_protos
    out = [("transformer", k, s) for k, s in transformer_shapes(H).items()]
    out += [("gen", k, s) for k, s in gen_shapes(H).items()]
    out += [("disc", k, s) for k, s in disc_shapes(H).items()]
    out += [("prototypes", "prototypes", (K, PROTO_DIM))]
    return out


def pack_blob(weights, H):
    """Concatenate a weight set into the float64 blob of ``pgp_load_weights``
    (PreGAN+ Transformer set, or PreGAN FPE set when ``weights`` has ``fpe``)."""
    K = np.asarray(weights["prototypes"]).shape[0]
    parts = []
    layout = fpe_blob_layout(H) if "fpe" in weights else blob_layout(H, K)
    for sec, name, shp in layout:
        a = np.asarray(weights[sec] if sec == "prototypes" else weights[sec][name],
                       dtype=np.float64)
        if a.shape != tuple(shp):
            raise ValueError(f"{sec}/{name}: shape {a.shape} != {shp}")
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def blob_size(H, n_protos=None):
    return sum(int(np.prod(s)) for _, _, s in blob_layout(H, n_protos))


def positional_encoding(d_model, max_len=3):
    """``models.py:297-307`` buffer, computed in fp32 as the reference does."""
    position = np.arange(0, max_len, dtype=np.float32)[:, None]
    div = np.exp(np.arange(0, d_model, 2, dtype=np.float32)
                 * np.float32(-np.log(10000.0) / d_model)).astype(np.float32)
    pe = np.zeros((max_len, d_model), dtype=np.float32)
    pe[:, 0::2] = np.sin(position * div)
    pe[:, 1::2] = np.cos(position * div)
    return pe.astype(np.float64)[:, None, :]


def synth_weights(H, seed=0):
    """Seeded weights for the H-generic model (uniform +-1/sqrt(fan_in), like
    torch's Linear default; LayerNorm gamma around 1; prototypes U(0,1) as
    ``models.py:373-374``).  Values are rounded to fp32-representable doubles so
    an fp32 kernel and an fp64 reference start from the same numbers."""
    if H % 2:
        raise ValueError("H must be even (d_model = H is split over 2 heads)")
    rng = np.random.Generator(np.random.PCG64(seed))

    def fill(shapes, sec):
        out = {}
        for name, shp in shapes.items():
            if name == "pos_encoder.pe":
                out[name] = positional_encoding(H, shp[0])
                continue
            if name.endswith("norm1.weight") or name.endswith("norm2.weight"):
                a = 1.0 + 0.1 * rng.uniform(-1, 1, size=shp)
            elif name.endswith("norm1.bias") or name.endswith("norm2.bias"):
                a = 0.1 * rng.uniform(-1, 1, size=shp)
            else:
                fan_in = shp[1] if len(shp) == 2 else shapes[name.replace("bias", "weight")][1]
                bound = 1.0 / np.sqrt(fan_in)
                a = rng.uniform(-bound, bound, size=shp)
            out[name] = a.astype(np.float32).astype(np.float64)
        return out

    w = {
        "transformer": fill(transformer_shapes(H), "t"),
        "gen": fill(gen_shapes(H), "g"),
        "disc": fill(disc_shapes(H), "d"),
    }
    w["prototypes"] = rng.uniform(0, 1, size=(H, PROTO_DIM)).astype(np.float32).astype(np.float64)
    return w


def torch_default_weights(H, seed=0):
    """A new model as the reference's constructors initialise it (load_model
    without a checkpoint, utils.py:76-78): nn.Linear weights and biases
    U(+-1/sqrt(fan_in)) (kaiming_uniform(a=sqrt(5)) and its bias rule);
    LayerNorm gamma 1, beta 0; nn.MultiheadAttention in_proj xavier_uniform
    (bound sqrt(6 / (d + 3d))), in_proj_bias and out_proj.bias 0, out_proj.weight
    the Linear rule; TransformerEncoder deep-copies its layer, so every layer
    starts from layer 0's values; prototypes U(0,1) (torch.rand, models.py:373).
    The distributions are torch's; the draws are numpy's (seeded), so the values
    are not torch's own (parity unpinned: only the offline-training fallback
    uses them).  fp32-representable doubles, as synth_weights."""
    if H % 2:
        raise ValueError("H must be even (d_model = H is split over 2 heads)")
    rng = np.random.Generator(np.random.PCG64(seed))

    def lin(shapes, name):
        shp = shapes[name]
        fan_in = shp[1] if len(shp) == 2 else shapes[name.replace("bias", "weight")][1]
        b = 1.0 / np.sqrt(fan_in)
        return rng.uniform(-b, b, size=shp)

    def fill(shapes):
        out = {}
        for name, shp in shapes.items():
            if name == "pos_encoder.pe":
                out[name] = positional_encoding(H, shp[0])
                continue
            if ".layers." in name and not name.startswith("transformer_encoder.layers.0."):
                continue   # cloned below
            if name.endswith(("norm1.weight", "norm2.weight")):
                a = np.ones(shp)
            elif name.endswith(("norm1.bias", "norm2.bias", "in_proj_bias", "out_proj.bias")):
                a = np.zeros(shp)
            elif name.endswith("in_proj_weight"):
                b = np.sqrt(6.0 / (shp[0] + shp[1]))
                a = rng.uniform(-b, b, size=shp)
            else:
                a = lin(shapes, name)
            out[name] = np.asarray(a, dtype=np.float32).astype(np.float64)
        for name in shapes:
            if ".layers." in name and name not in out:
                out[name] = out["transformer_encoder.layers.0." + name.split(".", 3)[3]].copy()
        return {k: out[k] for k in shapes}

    w = {"transformer": fill(transformer_shapes(H)), "gen": fill(gen_shapes(H)), "disc": fill(disc_shapes(H))}
    w["prototypes"] = rng.uniform(0, 1, size=(H, PROTO_DIM)).astype(np.float32).astype(np.float64)
    return w


def torch_default_fpe_weights(H=16, seed=0):
    """A new PreGAN model as its constructors initialise it (load_model without
    a checkpoint): nn.GRU every parameter U(+-1/sqrt(hidden = 3)); nn.Linear
    U(+-1/sqrt(fan_in)) for weights and biases (GAT fc / attn_fc have no bias,
    dlutils.py:300-301); nn.MultiheadAttention in_proj xavier_uniform, in_proj
    and out_proj biases 0, out_proj.weight the Linear rule; prototypes U(0,1)
    (torch.rand, models.py:62); Gen / Disc nn.Linear.  torch's distributions,
    numpy's draws (parity unpinned for the values themselves)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {"fpe": {}, "gen": {}, "disc": {}}
    for sec, shapes in (("fpe", fpe_shapes(H)), ("gen", gen_shapes(H)), ("disc", disc_shapes(H))):
        for name, shp in shapes.items():
            if name.startswith("gru."):
                a = rng.uniform(-1, 1, size=shp) / np.sqrt(3.0)
            elif name.endswith(("in_proj_bias", "out_proj.bias")):
                a = np.zeros(shp)
            elif name.endswith("in_proj_weight"):
                b = np.sqrt(6.0 / (shp[0] + shp[1]))
                a = rng.uniform(-b, b, size=shp)
            else:
                fan_in = shp[1] if len(shp) == 2 else shapes[name.replace("bias", "weight")][1]
                a = rng.uniform(-1, 1, size=shp) / np.sqrt(fan_in)
            out[sec][name] = np.asarray(a, dtype=np.float32).astype(np.float64)
    out["prototypes"] = rng.uniform(0, 1, size=(FPE_PROTOS, PROTO_DIM)).astype(np.float32).astype(np.float64)
    return out


def weights_checksum(weights):
    h = 0.0
    for sec in ("transformer", "gen", "disc"):
        for k in sorted(weights[sec]):
            a = np.asarray(weights[sec][k], dtype=np.float64).reshape(-1)
            h += float(np.dot(a, np.cos(np.arange(a.size) * 0.001)))
    return h + float(np.asarray(weights["prototypes"]).sum())


_BUFFERS = {"transformer": ("pos_encoder.pe",), "fpe": (), "gen": (), "disc": ()}   # state_dict entries that are not parameters


def load_reference_checkpoints(model_dir, env_name="simulator", H=16, encoder="Transformer", with_state=False,
                               gan_fresh=None):
    """Read ``{env}_Transformer_{H}.ckpt``/``Gen``/``Disc`` from a COSCO tree
    (``checkpointsplus/``; format ``utils.py:53-58``) with the safe loader.

    with_state=True also returns ``extra``, the training state ``load_model`` /
    ``load_gan`` restore (``utils.py:60-84``) in the packaged-npz key format the
    Trainer reads: AdamW ``opt/{sec}/{name}/exp_avg|exp_avg_sq|step`` (the
    optimizer state is keyed by parameter index, i.e. ``named_parameters``
    order = the state_dict order without buffers), ``meta/{sec}/epoch`` and the
    Gen checkpoint's ``accuracy_list`` (the one PreGANPlusRecovery keeps,
    ``PreGANPlus.py:32-34``) as ``meta/gen/accuracy_list`` (flat) +
    ``meta/gen/accuracy_list_lens``.

    ``gan_fresh`` ({"gen": ..., "disc": ...} weights of a new GAN, or a
    callable returning them, called only when needed): a Gen or
    Disc checkpoint that is absent is replaced by that new model, as
    ``load_gan`` -> ``load_model`` creates one (utils.py:76-78, 81-84: Gen
    epoch -1 and an empty accuracy_list, no optimizer state); without it an
    absent file raises."""
    def path(name):
        return os.path.join(model_dir, f"{env_name}_{name}_{H}.ckpt")

    t = _safe_load(path(encoder))
    new_model = {"epoch": -1, "accuracy_list": [], "model_state_dict": None}
    g, d = ({**new_model, "fresh": n} if gan_fresh is not None and not os.path.exists(path(n)) else _safe_load(path(n))
            for n in ("Gen", "Disc"))
    tsec = "fpe" if encoder == "FPE" else "transformer"
    if g.get("fresh") or d.get("fresh"):
        gan_fresh = gan_fresh() if callable(gan_fresh) else gan_fresh
    sd = lambda ck, sec: (dict(gan_fresh[sec]) if ck.get("fresh") else _conv_sd(ck["model_state_dict"]))
    weights = {
        tsec: _conv_sd(t["model_state_dict"]),
        "gen": sd(g, "gen"),
        "disc": sd(d, "disc"),
        "prototypes": np.stack([p.detach().cpu().numpy() for p in t["model_prototypes"]]),
        "meta": {"epoch": t["epoch"], "gan_epoch": g["epoch"]},
    }
    if not with_state:
        return weights
    extra = {}
    for sec, ck in ((tsec, t), ("gen", g), ("disc", d)):
        extra.update({f"meta/{sec}/epoch": np.int64(-1)} if ck.get("fresh") else _ck_state(sec, ck))
    extra.update(accuracy_list_to_arrays(g["accuracy_list"], "meta/gen/accuracy_list"))
    # the encoder checkpoint's own accuracy_list (train_model's, PreGANPlus.py:41-49): kept
    # apart so an explicit full save writes the encoder checkpoint as load_model read it
    extra.update(accuracy_list_to_arrays(t["accuracy_list"], f"meta/{tsec}/accuracy_list"))
    return weights, extra


def _safe_load(path):
    import torch
    sg = [(np._core.multiarray.scalar, "numpy.core.multiarray.scalar"), np.dtype, np.dtypes.Float64DType]
    with torch.serialization.safe_globals(sg):
        return torch.load(path, weights_only=True)


def _conv_sd(sd):
    return {k: v.detach().cpu().numpy().astype(np.float64) for k, v in sd.items()}


def _ck_state(sec, ck):
    """load_model's training state of one checkpoint (utils.py:70-77) in the
    packaged-npz key format: AdamW moments / steps per parameter, epoch."""
    extra = {}
    names = [k for k in ck["model_state_dict"] if k not in _BUFFERS[sec]]
    osd = ck["optimizer_state_dict"]
    idx = [i for grp in osd["param_groups"] for i in grp["params"]]
    if len(idx) != len(names):
        raise ValueError(f"{sec}: {len(idx)} optimizer params vs {len(names)} state_dict parameters")
    for i, name in zip(idx, names):
        s = osd["state"].get(i)
        if not s:
            continue
        extra[f"opt/{sec}/{name}/exp_avg"] = s["exp_avg"].detach().cpu().numpy().astype(np.float64)
        extra[f"opt/{sec}/{name}/exp_avg_sq"] = s["exp_avg_sq"].detach().cpu().numpy().astype(np.float64)
        extra[f"opt/{sec}/{name}/step"] = np.float64(float(s["step"]))
    extra[f"meta/{sec}/epoch"] = np.int64(ck["epoch"])
    return extra


def load_gan_checkpoints(model_dir, env_name="simulator", H=16):
    """load_gan (utils.py:81-84) alone: Gen / Disc weights and their training
    state from ``{env}_Gen_{H}.ckpt`` / ``{env}_Disc_{H}.ckpt`` (the files
    save_gan rewrites every call), or None when either is absent."""
    paths = [os.path.join(model_dir, f"{env_name}_{n}_{H}.ckpt") for n in ("Gen", "Disc")]
    if not all(os.path.exists(p) for p in paths):
        return None
    g, d = (_safe_load(p) for p in paths)
    weights = {"gen": _conv_sd(g["model_state_dict"]), "disc": _conv_sd(d["model_state_dict"])}
    extra = dict(_ck_state("gen", g), **_ck_state("disc", d))
    extra.update(accuracy_list_to_arrays(g["accuracy_list"], "meta/gen/accuracy_list"))
    return weights, extra


def accuracy_list_to_arrays(acc, key):
    """A checkpoint accuracy_list (tuples of 2 or 4 numbers) as npz arrays."""
    vals = [np.asarray([float(v) for v in (e if isinstance(e, (tuple, list)) else (e,))]) for e in acc]
    flat = np.concatenate(vals) if vals else np.zeros(0)
    return {key: flat, key + "_lens": np.array([len(v) for v in vals], dtype=np.int64)}


def accuracy_list_from_arrays(extra, key):
    if key not in extra:
        return []
    flat, lens = np.asarray(extra[key], np.float64), np.asarray(extra[key + "_lens"], np.int64)
    out, o = [], 0
    for n in lens:
        out.append(tuple(float(v) for v in flat[o:o + n]))
        o += n
    return out


def save_npz(path, weights, extra=None):
    flat = {}
    for sec in ("transformer", "fpe", "gen", "disc"):
        for k, v in weights.get(sec, {}).items():
            flat[f"{sec}/{k}"] = np.asarray(v, dtype=np.float64)
    flat["prototypes"] = np.asarray(weights["prototypes"], dtype=np.float64)
    for k, v in (extra or {}).items():
        flat[k] = v
    np.savez_compressed(path, **flat)


def load_npz(path):
    z = np.load(path, allow_pickle=False)
    w = {"transformer": {}, "fpe": {}, "gen": {}, "disc": {}}
    extra = {}
    for k in z.files:
        sec = k.split("/", 1)[0]
        if sec in w:
            w[sec][k.split("/", 1)[1]] = z[k]
        elif k == "prototypes":
            w["prototypes"] = z[k]
        else:
            extra[k] = z[k]
    for sec in ("transformer", "fpe"):
        if not w[sec]:
            del w[sec]
    return w, extra
