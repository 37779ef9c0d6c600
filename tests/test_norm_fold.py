"""The histogram path's folded additive normalisation (NORM 3 in csrc/sg_stack_hist.hip).

The reference normalises a sample as round_to_WORD(v * scale - offset)
(src/stacking/stacking.c:1635-1652, round_to_WORD src/core/utils.c:68-74): two double
roundings, then (WORD)(x + 0.5) for 0 < x <= 65535.  When c = offset - 0.5 is exact, the
kernel computes trunc(v * scale - c) instead (one double add per sample less).  The host
enables the fold only when the TwoSum error of offset - 0.5 is zero (csrc/sg_api.cpp); this
test checks the equality over every u16 sample value for random and adversarial offsets
(half-integers and their neighbours), and the host's exactness test itself.
"""
import numpy as np

V = np.arange(65536, dtype=np.float64)


def reference(scale, offset):
    x = V * scale - offset
    return np.where(x <= 0, 0, np.where(x > 65535, 65535, np.trunc(x + 0.5))).astype(np.int64)


def folded(scale, c):
    z = V * scale - c
    return np.clip(np.trunc(np.maximum(z, 0.0)), 0, 65535).astype(np.int64)


def fold_exact(b):
    """the host's test: TwoSum error of b - 0.5 is zero"""
    c = b - 0.5
    bb = c - b
    return ((b - (c - bb)) + (-0.5 - bb)) == 0.0


def test_fold_equals_reference_rounding():
    rng = np.random.default_rng(7)
    tested = 0
    for i in range(600):
        scale = rng.uniform(0.5, 2.0) if i % 3 else 1.0 + float(rng.integers(-3, 4)) * 2.0 ** -int(rng.integers(1, 30))
        kind = i % 5
        if kind == 0:
            b = rng.uniform(-200, 200)
        elif kind == 1:
            b = float(rng.integers(-200, 200)) + 0.5
        elif kind == 2:
            b = float(rng.integers(-200, 200)) + 0.5 + float(rng.choice([-1, 1])) * 2.0 ** -int(rng.integers(20, 52))
        elif kind == 3:
            b = rng.uniform(-2000, 2000) * 2.0 ** -int(rng.integers(0, 12))
        else:
            b = float(np.nextafter(float(rng.integers(-300, 300)) + 0.5, float(rng.choice([-1e9, 1e9]))))
        if not fold_exact(b):
            continue
        tested += 1
        assert np.array_equal(reference(scale, b), folded(scale, b - 0.5)), (scale, b)
    assert tested > 500


def test_fold_exactness_check():
    assert fold_exact(123.25) and fold_exact(-7.0) and fold_exact(0.5)
    assert not fold_exact(2.0 ** -60)          # 2^-60 - 0.5 needs 60 bits
    assert not fold_exact(1e-30)
