"""GPU checks of the online interval's composition (bench.py --config loop,
DESIGN.md §11): staged forward, GAN step with device labels, weight sync.

recover_decision runs after train_gan with the UPDATED GAN on the embedding
computed BEFORE training (PreGANPlus.py:130-136).  The loop does this with
pgp_forward_stage 0-2, a training step, DecisionModel.load_master and stage 3.
With only a GAN step (encoder weights unchanged), that must equal a fresh model
built from the trained weights and run end to end: same kernels, same inputs,
bit-identical outputs."""
import numpy as np
import pytest
import torch

from preganplus_amd import simulate as SIM
from preganplus_amd import train as TR
from preganplus_amd import weights as W
from preganplus_amd.model import DecisionModel, to_numpy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,B", [(16, 64), (50, 24)])
def test_staged_forward_after_gan_step_equals_fresh_model(H, B):
    if H == 16:
        w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    else:
        w = W.synth_weights(H, seed=12)
    dev = torch.device("cuda")
    rng = np.random.Generator(np.random.PCG64(H + B))
    x = rng.uniform(0, 0.6, size=(B, 3, 3 * H))
    x = np.where(rng.uniform(size=x.shape) < 0.05, rng.uniform(0.9, 1.3, size=x.shape), x)
    xt = torch.tensor(x, dtype=torch.float32, device=dev)
    s = np.zeros((B, H, H), np.float32)
    s[np.arange(B)[:, None], np.arange(H)[None, :], rng.integers(0, H, (B, H))] = 1.0
    st = torch.tensor(s, device=dev)
    model = DecisionModel(H, w, device=dev)
    tr = TR.Trainer(H, w, max_batch=B)
    model.load_master(tr.P, model.prototypes)  # pack from the fp32 master, as after every interval
    out = model.alloc_outputs(B)
    for stage in (0, 1, 2):
        model.forward(xt, st, out=out, stage=stage)
    emb = torch.where(out["logits"][..., 1:2] > out["logits"][..., 0:1], out["protos"], 0.0)
    TR.train_gan_batched(tr, SIM.Simulation(H), SIM.synth_envs(B, H, seed=3), emb, st)
    model.load_master(tr.P, model.prototypes)
    model.forward(xt, st, out=out, stage=3)
    got = to_numpy(out)

    w2 = tr.weights_numpy()
    w2["prototypes"] = np.asarray(w["prototypes"])
    fresh = to_numpy(DecisionModel(H, w2, device=dev).forward(xt, st))
    for k in ("logits", "protos", "cls", "any", "probs", "keep", "final_target", "gen_target"):
        assert np.array_equal(got[k], fresh[k]), k
    # and the GAN really moved: the pre-training weights give other probabilities
    before = DecisionModel(H, w, device=dev)
    before.load_master(TR.Trainer(H, w, max_batch=B).P, model.prototypes)
    assert not np.array_equal(to_numpy(before.forward(xt, st))["probs"], got["probs"])
