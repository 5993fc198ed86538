"""K5 (pgp_migrations) vs the oracle's recover_decision assembly
(PreGANPlus.py:87-105): bit-exact moves / hosts_from and the same returned
decision list, over random placements with unplaced (-1) containers, both keep
outcomes, H in {16, 50}, and an empty batch."""
import numpy as np
import pytest
import torch

from oracle import pregan_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H", [16, 50])
def test_migrations_match_oracle(H):
    from preganplus_amd.model import assemble_decision, migrations
    rng = np.random.Generator(np.random.PCG64(H))
    B = 3000
    keep = (rng.uniform(size=B) < 0.3).astype(np.int32)
    tgt = rng.integers(0, H, size=(B, H)).astype(np.int32)
    cur = rng.integers(-1, H, size=(B, H)).astype(np.int32)
    cur[5] = -1                                  # nothing placed
    tgt[6] = cur[6].clip(0)                      # every placed container already on target
    keep[5:7] = 0
    d = lambda a: torch.tensor(a, device="cuda")
    mv, hf = migrations(d(keep), d(tgt), d(cur))
    mv, hf = mv.cpu().numpy(), hf.cpu().numpy()
    for b in range(B):
        orig = [(int(c), int(rng.integers(0, H))) for c in rng.permutation(H)[:H // 2]]
        containers = [(c, int(cur[b, c])) for c in range(H) if cur[b, c] >= 0]
        ref_list, ref_hf = O.recover_decision_list(bool(keep[b]), tgt[b], containers, H, orig)
        if keep[b]:
            assert (mv[b] == -1).all() and (hf[b] == 0).all()
            continue
        got_list = assemble_decision(orig, mv[b], cur[b])
        assert got_list == ref_list, b
        assert hf[b].tolist() == ref_hf, b


def test_migrations_empty_batch():
    from preganplus_amd.model import migrations
    z = torch.zeros((0, 16), dtype=torch.int32, device="cuda")
    mv, hf = migrations(torch.zeros(0, dtype=torch.int32, device="cuda"), z, z)
    assert mv.shape == (0, 16) and hf.shape == (0, 16)


def test_migrations_out_of_range_host_is_unplaced():
    """A current-host index outside [0, C) never writes through: the
    container is treated as unplaced, exactly like -1."""
    from preganplus_amd.model import migrations
    H = 16
    d = lambda a: torch.tensor(np.asarray(a, dtype=np.int32), device="cuda")
    cur = np.array([[3, 16, 1000, -7, 5] + [2] * (H - 5), [-1] * H])
    tgt = np.zeros((2, H), dtype=np.int32)
    ref = cur.copy()
    ref[(ref < 0) | (ref >= H)] = -1
    mv, hf = migrations(d([0, 0]), d(tgt), d(cur))
    mv2, hf2 = migrations(d([0, 0]), d(tgt), d(ref))
    assert torch.equal(mv, mv2) and torch.equal(hf, hf2)
    assert mv[0, 1].item() == -1 and mv[0, 2].item() == -1 and int(hf[0].sum().item()) == 3


def test_embedding_matches_reference_rule():
    """pgp_embedding = run_model's embedding line (PreGANPlus.py:129): the host's
    prototype where argmax(logits) == 1 (torch.argmax: ties -> 0), else zeros;
    bit-exact, ties and ragged batches included."""
    import torch
    from preganplus_amd.model import embedding
    rng = np.random.Generator(np.random.PCG64(5))
    for B, H in ((1, 16), (77, 50), (1000, 8)):
        lg = rng.standard_normal((B, H, 2)).astype(np.float32)
        lg[::3, ::2, 1] = lg[::3, ::2, 0]                      # ties
        pr = rng.uniform(size=(B, H, 2)).astype(np.float32)
        want = np.where((lg[..., 1] > lg[..., 0])[..., None], pr, 0.0).astype(np.float32)
        got = embedding(torch.tensor(lg, device="cuda"), torch.tensor(pr, device="cuda")).cpu().numpy()
        assert np.array_equal(got, want)
