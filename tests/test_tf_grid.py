"""The fused tuning launches' workgroup count (pgp_tunef.hip tf_grid_for,
mirrored by roofline.tf_grid for the bench's CU report): the fewest workgroups
whose longest wave has as many units as on the whole budget."""
from preganplus_amd import roofline as R


def _longest(units, waves, grid):
    nw = grid * waves
    return units // nw + (1 if units % nw else 0)


def test_fewest_workgroups_same_longest_wave():
    for units in (1, 15, 992, 1024, 1030, 3200, 3219, 3541, 10_000):
        for waves in (4, 8):
            for reserve in (0, 8, 200):
                g = R.tf_grid(units, waves, 256, reserve)
                gmax = max(1, min(256 - min(reserve, 128), -(-units // waves)))
                assert 1 <= g <= gmax
                assert _longest(units, waves, g) == _longest(units, waves, gmax)
                if g > 1:   # one workgroup fewer would lengthen the longest wave
                    assert _longest(units, waves, g - 1) > _longest(units, waves, gmax)


def test_c3_shapes():
    assert R.tf_grid(3200, 4, 256, 8) == 200      # H = 50, 1,024 windows: the backward
    assert R.tune_fused_grids(50, 1030, 1133, 256, 8) == [222, 222, 202, 202, 202, 202]
    assert R.tune_fused_grids(16, 1030, 1133, 256, 8) == [142, 142, 129, 129, 129, 129]
