"""C5 streamed (preganplus_amd/fleet.py): cell-window chunks copied in from
pinned host memory, double-buffered against the kernels, decisions copied out.
The streamed outputs must be bitwise those of the resident launch on the same
chunk, and a streamed full-size chunk passes the census against the fp64
oracle (tests/census.py)."""
import numpy as np
import pytest
import torch

from preganplus_amd import weights as W

pytestmark = pytest.mark.gpu


def _model():
    from preganplus_amd.model import DecisionModel
    w, _ = W.load_npz("preganplus_amd/data/simulator_16.npz")
    return w, DecisionModel(16, w, device="cuda")


def _chunk(B, H, seed):
    from tests.test_gpu_parity import _c2_torch
    x, s = _c2_torch(B, H, seed=seed)
    return x, s, s.argmax(dim=-1)


def test_schedule_onehot_kernel():
    from preganplus_amd.fleet import schedule_onehot
    for H in (16, 50):
        rng = np.random.Generator(np.random.PCG64(H))
        idx = rng.integers(0, H + 3, size=(777, H)).astype(np.uint8)   # >= H: an unplaced row
        got = schedule_onehot(torch.tensor(idx, device="cuda"), torch.full((777, H, H), 7.0, device="cuda"), H)
        ref = (idx[..., None] == np.arange(H)).astype(np.float32)
        assert np.array_equal(got.cpu().numpy(), ref)
    with pytest.raises(ValueError):
        schedule_onehot(torch.zeros((4, 16), dtype=torch.int32, device="cuda"),
                        torch.zeros((4, 16, 16), device="cuda"), 16)


def test_streamed_equals_resident():
    """5 chunks of 4,096 cell-windows cycled over 3 pinned sources: every
    output of every chunk bitwise equal to the resident forward of its source."""
    from preganplus_amd.fleet import ALL_KEYS, FleetStreamer, pinned_chunk
    from preganplus_amd.model import to_numpy
    w, m = _model()
    B, H = 4096, 16
    chunks = [_chunk(B, H, 500 + k) for k in range(3)]
    srcs = [pinned_chunk(x, i) for x, _, i in chunks]
    fs = FleetStreamer(m, B, keys=ALL_KEYS)
    dest = fs.host_outputs(5)
    fs.run(srcs, 5, dest)
    torch.cuda.synchronize()
    for i in range(5):
        x, s, _ = chunks[i % 3]
        ref = to_numpy(m.forward(x, s))
        torch.cuda.synchronize()
        for k in ALL_KEYS:
            assert np.array_equal(dest[i][k].numpy(), ref[k]), (i, k)


@pytest.mark.timeout(600)
def test_streamed_chunk_census():
    """One full C5 chunk (262,144 cell-windows, shipped H=16 weights) through
    the streaming pipeline (two chunks streamed, the second checked), every
    window compared with the fp64 oracle as in the resident census."""
    from preganplus_amd.fleet import ALL_KEYS, FleetStreamer, pinned_chunk
    from tests import census as CE
    from tests import decision_bounds as DB
    w, m = _model()
    B, H = 262144, 16
    a = _chunk(B, H, 901)
    b = _chunk(B, H, 902)
    srcs = [pinned_chunk(a[0], a[2]), pinned_chunk(b[0], b[2])]
    fs = FleetStreamer(m, B, keys=ALL_KEYS)
    dest = fs.host_outputs(2)
    fs.run(srcs, 2, dest)
    torch.cuda.synchronize()
    got = {k: v.numpy() for k, v in dest[1].items()}
    x32 = b[0].cpu().numpy()
    sidx = b[2].cpu().numpy()
    del a, b
    st, worst = CE.run(w, x32, sidx, got, log=print)
    print("STREAMED CENSUS", st["windows"], worst)
    assert worst["logits"] <= 1.0 and worst["protos"] <= 1.0 and worst["probs"] <= 1.0, worst
    assert not DB.violations(st), st
    assert st["windows"] == B
    for kind in ("anomaly", "any", "class", "keep", "final"):
        assert st[kind]["mismatch"] == 0, (kind, st[kind])
    assert st["gen"]["mismatch"] <= 8, st["gen"]
