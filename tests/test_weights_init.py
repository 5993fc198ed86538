"""weights.torch_default_weights (the new-model fallback of load_models,
utils.py:76-78): the same constants and bounds as torch's own module
constructors for the reference's Transformer_H parts (nn.Linear,
nn.LayerNorm, nn.MultiheadAttention inside nn.TransformerEncoderLayer, the
deep-copied layers of nn.TransformerEncoder), Gen and Disc."""
import numpy as np
import torch

from preganplus_amd import weights as W


def _torch_layer(H):
    torch.manual_seed(0)
    layer = torch.nn.TransformerEncoderLayer(d_model=H, nhead=2, dim_feedforward=64, dropout=0.1)
    return dict(torch.nn.TransformerEncoder(layer, num_layers=2, enable_nested_tensor=False).named_parameters())


def test_torch_default_weights_match_module_constructors():
    H = 16
    w = W.torch_default_weights(H, seed=3)
    t = w["transformer"]
    ref = _torch_layer(H)
    for name, p in ref.items():
        ours = t["transformer_encoder." + name]
        tv = p.detach().double().numpy()
        assert ours.shape == tv.shape, name
        if np.all(tv == tv.flat[0]):          # constant init in torch (LayerNorm 1/0, MHA biases 0)
            assert np.all(ours == tv.flat[0]), name
        else:                                 # same uniform bound
            fan_in, fan_out = tv.shape[1] if tv.ndim == 2 else None, tv.shape[0]
            if name.endswith("in_proj_weight"):
                bound = np.sqrt(6.0 / (fan_in + fan_out))
            else:
                wname = name.replace("bias", "weight")
                bound = 1.0 / np.sqrt(ref[wname].shape[1])
            assert np.abs(tv).max() <= bound and np.abs(ours).max() <= bound * (1 + 1e-6), name
            assert np.abs(ours).max() > 0.5 * bound, name
    # TransformerEncoder deep-copies its layer: both layers start equal
    for k, v in t.items():
        if k.startswith("transformer_encoder.layers.1."):
            np.testing.assert_array_equal(v, t[k.replace("layers.1.", "layers.0.")])
    assert set(t) == set(W.transformer_shapes(H))
    assert np.all((w["prototypes"] >= 0) & (w["prototypes"] < 1))
    for sec, shapes in (("gen", W.gen_shapes(H)), ("disc", W.disc_shapes(H))):
        for k, shp in shapes.items():
            fan_in = shapes[k.replace("bias", "weight")][1]
            assert w[sec][k].shape == shp and np.abs(w[sec][k]).max() <= 1 / np.sqrt(fan_in) * (1 + 1e-6)
