"""CPU: the ORB spec restatement (oracle/sfm_oracle_orb.c) against independent checks — the
exact rotation rounding vs rational arithmetic, FAST / Harris on constructed patterns, the level
budget of OpenCV's ORB (code/feature_matching.py:42 defaults), the BRIEF pattern = OpenCV's learned
bit_pattern_31_ (scikit-image's copy of the table, when present here)."""
import math
import os
from fractions import Fraction

import numpy as np

import oracle as O
import synth


def test_round_div_is_exact():
    rng = np.random.default_rng(0)
    for _ in range(3000):
        m10, m01 = (int(v) for v in rng.integers(-3_000_000, 3_000_000, 2))
        R2 = m10 * m10 + m01 * m01
        if R2 == 0:
            continue
        n = int(rng.integers(-13, 14)) * m10 - int(rng.integers(-13, 14)) * m01
        k = O.orb_round_div(n, R2)
        # k = floor(n / sqrt(R2) + 1/2)  <=>  (2k - 1) sqrt(R2) <= 2n < (2k + 1) sqrt(R2)
        lo, hi = 2 * k - 1, 2 * k + 1
        cmp = lambda B, A: (B <= 0 <= A) or (B >= 0 and A >= 0 and B * B * R2 <= A * A) or (
            B < 0 and A < 0 and B * B * R2 >= A * A)
        assert cmp(lo, 2 * n) and not cmp(hi, 2 * n)
        assert abs(k - n / math.sqrt(R2)) <= 0.5 + 1e-9


def test_level_budget_and_sizes():
    Wl, Hl, sc, nl = O.orb_levels(1920, 1080)
    assert nl.sum() == 500 and list(nl[:3]) == [109, 90, 75]
    assert list(Wl[:4]) == [1920, 1600, 1333, 1111] and list(Hl[:4]) == [1080, 900, 750, 625]
    np.testing.assert_allclose(sc, 1.2 ** np.arange(8))


def test_fast_score_and_harris_on_a_corner():
    L = np.full((80, 80), 50, np.uint8)
    L[40:, 40:] = 200                       # bright quadrant: corner at (40, 40)
    assert O.orb_fast_score(L, 40, 40) > 20 and O.orb_fast_score(L, 60, 60) == 0
    assert O.orb_fast_score(L, 60, 40) == 0  # straight edge: no 9-arc of brighter pixels
    assert O.orb_harris(L, 40, 40) > 0 > O.orb_harris(L, 60, 40)
    assert O.orb_harris(L, 20, 20) == 0


def test_resize_and_blur_keep_constants():
    c = np.full((90, 120), 77, np.uint8)
    assert (O.orb_resize(c, 75, 100) == 77).all() and (O.orb_blur(c) == 77).all()


SKIMAGE_POS = "/opt/conda/lib/python3.9/site-packages/skimage/feature/orb_descriptor_positions.txt"


def test_pattern_is_opencv_bit_pattern_31():
    p = O.orb_pattern()
    assert p.shape == (256, 4) and p.min() >= -13 and p.max() <= 12
    # OpenCV's first and last entries of bit_pattern_31_ (x1, y1, x2, y2)
    assert p[:4].tolist() == [[8, -3, 9, 5], [4, 2, 7, -12], [-11, 9, -8, 2], [7, -12, 12, -13]]
    assert not ((p[:, 0] == p[:, 2]) & (p[:, 1] == p[:, 3])).any()
    if os.path.exists(SKIMAGE_POS):  # this container: the generated header equals the source table
        ref = np.loadtxt(SKIMAGE_POS).astype(np.int32)
        np.testing.assert_array_equal(p, ref)


def test_orb_oracle_end_to_end():
    img = synth.make_image(240, 320, seed=2)
    kp, desc, lc = O.orb(img)
    assert len(kp) == lc.sum() > 100
    assert (kp[:, 0] >= 0).all() and (kp[:, 0] < 320).all() and (kp[:, 1] < 240).all()
    assert (np.diff(kp[:, 5]) >= 0).all()   # level order
