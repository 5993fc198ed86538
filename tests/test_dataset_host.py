"""The plugin's host-side on-the-fly dataset (train.form_test_dataset,
convert_to_windows, percentile_linear; utils.py:7-24) is vectorised; it must
stay bit-identical to the loop form over np.percentile that mirrors the
reference line by line (ties, constant columns and short series included)."""
import numpy as np
import pytest

from preganplus_amd import train as TR


def loop_form(data):
    anomaly_per_dim = data > np.percentile(data, TR.PERCENTILES, axis=0)
    which, anydim = [], []
    for i in range(0, data.shape[1], 3):
        which.append(np.argmax(data[:, i:i + 3] + 0, axis=1))
        anydim.append(np.logical_or.reduce(anomaly_per_dim[:, i:i + 3], axis=1))
    return np.stack(anydim, axis=1) + 0, np.stack(which, axis=1)


def loop_windows(data, n_window=3):
    out = []
    for i in range(data.shape[0]):
        if i >= n_window:
            out.append(data[i - n_window:i])
        else:
            out.append(np.concatenate([np.repeat(data[0:1], n_window - i, axis=0), data[0:i]]))
    return np.stack(out)


@pytest.mark.parametrize("R", [1, 2, 3, 4, 10, 16, 101])
def test_dataset_matches_loop_form(R):
    rng = np.random.default_rng(R)
    for t in range(60):
        H = int(rng.choice([8, 16, 50]))
        d = rng.random((R, 3 * H))
        if t % 3 == 0:
            d = np.round(d * 4) / 4  # ties
        if t % 7 == 0:
            d[:, :6] = 0.5  # constant columns
        a1, w1 = loop_form(d)
        a2, w2 = TR.form_test_dataset(d)
        assert np.array_equal(a1, a2) and np.array_equal(w1, w2)
        assert a1.dtype == a2.dtype and w1.dtype == w2.dtype
        assert np.array_equal(np.percentile(d, TR.PERCENTILES, axis=0), TR.percentile_linear(d, TR.PERCENTILES))
        assert np.array_equal(loop_windows(d), TR.convert_to_windows(d))
