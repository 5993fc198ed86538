"""Compare the plugin's tuning with host vs device custom_loss bookkeeping
(bit-level), and run-to-run determinism of each."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from preganplus_amd import train as TR, weights as W
from preganplus_amd.recovery import PreGANPlusRecovery
from tests.test_train_oracle_golden import fake_env

new_backprop = TR.backprop


def host_backprop(tr, st, wins, anom, cls):
    st.num_zero, st.num_ones = 1, 1
    losses = []
    for i in range(wins.shape[0]):
        logits, protos = tr.tune_forward(torch.as_tensor(wins[i:i + 1], dtype=torch.float32))
        mult, tgt, aloss, tloss = TR.loss_targets(logits[0].cpu().numpy(), protos[0].cpu().numpy(), anom[i], cls[i], st)
        tr.tune_backward(1, anom[i][None], mult[None], tgt[None])
        inactive = () if np.any(anom[i] > 0) else ("prototype_decoder.0.weight", "prototype_decoder.0.bias")
        tr.adam_step("transformer", inactive)
        losses.append((aloss, tloss))
    return losses


def run(bp):
    TR.backprop = bp
    w, extra = W.load_npz("preganplus_amd/data/simulator_16.npz")
    z = np.load("tests/golden/plugin_h16.npz")
    rec = PreGANPlusRecovery(16, "", training=True, weights=w, extra=extra)
    P = []
    for step in range(4):
        rec.setEnvironment(fake_env(z, step, extra["train_time_data"], z["schedule_series"]))
        rec.run_model(None, [tuple(x) for x in z[f"s{step}/decision_in"]])
        P.append(rec.trainer.P.cpu().numpy().copy())
    return P, rec.tune_state.protos.copy()


h1, ph1 = run(host_backprop)
h2, ph2 = run(host_backprop)
d1, pd1 = run(new_backprop)
d2, pd2 = run(new_backprop)
for s in range(4):
    print(f"step {s}: host-host {np.abs(h1[s]-h2[s]).max():.3e} dev-dev {np.abs(d1[s]-d2[s]).max():.3e} "
          f"host-dev {np.abs(h1[s]-d1[s]).max():.3e} n_diff {(h1[s]!=d1[s]).sum()}")
print("protos host-dev", np.abs(ph1 - pd1).max())
