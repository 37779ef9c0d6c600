"""Single-rounding / integer normalising loads of the histogram kernels (round 6).

The reference normalises a sample x of frame f in two or three double roundings
(src/stacking/stacking.c:1642-1651, round_to_WORD src/core/utils.c:68-74):
    additive        round_to_WORD(fl(x scale) - offset)
    multiplicative  round_to_WORD(fl(x scale) mul)
k_norm_fma_check (csrc/sg_stack_hist.hip) compares those, for every u16 x of every frame, with
one fma(x, a, b) per sample and lets the histogram kernels load through the fma only when no x of
any frame differs (sg_stack_stats.norm_fma = 1); additive normalisation with scale 1 (Siril's
ADDITIVE) also tries clamp(x - K, 0, 65535) with an integer K per frame (two packed saturating u16
ops per pixel pair, norm_fma = 2).  Otherwise the call keeps the reference's operations
(norm_fma = 0).  Either way the image and the counters equal the oracle.

The CPU test pins the premise of the fallback case: for the constructed coefficients the fma
really differs from the reference's roundings at one sample value (exact rational arithmetic,
CPython's correctly rounded Fraction -> float).
"""
from fractions import Fraction

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg


def _adversarial_frame_coeffs():
    """scale s and offset o (additive, offset - 0.5 exact) and a sample x0 whose reference value
    fl(fl(x0 s) - (o - 0.5)) truncates to k while fma(x0, s, -(o - 0.5)) truncates to k - 1:
    P = fl(x0 s) above the exact product, o - 0.5 = P - k, so the reference lands on k exactly and the
    exact x0 s - (o - 0.5) = k - (P - x0 s) lies just below it (resolved at k's small exponent)"""
    s = 1.0 + 3.3 * 2.0 ** -20
    for x0 in range(40000, 65536):
        P = x0 * s
        if Fraction(P) > Fraction(x0) * Fraction(s):
            k = 5
            c = P - k                       # exact: same binade as P, integer k
            o = c + 0.5                     # exact (0.5 is a multiple of c's spacing)
            assert o - 0.5 == c
            return s, o, x0, k
    raise AssertionError("no x0 found")


def _ref_trunc(x, s, c):
    """the kernels' NORM 3 form: trunc(fl(fl(x s) - c)), clamped like v_cvt_u32_f64 + the pack"""
    y = (x * s) - c
    return 0 if y <= 0 else min(int(y), 65535)


def _fma_trunc(x, s, c):
    y = float(Fraction(x) * Fraction(s) - Fraction(c))   # correctly rounded: one rounding
    return 0 if y <= 0 else min(int(y), 65535)


def test_adversarial_premise():
    s, o, x0, k = _adversarial_frame_coeffs()
    c = o - 0.5
    assert _ref_trunc(x0, s, c) == k
    assert _fma_trunc(x0, s, c) == k - 1
    # and the reference itself (round_to_WORD(fl(x s) - o)) agrees with the folded form there
    y = (x0 * s) - o
    assert (0 if y <= 0 else int(y + 0.5)) == k


@pytest.mark.gpu
@pytest.mark.parametrize("method,rejection", [(sg.MEAN, sg.SIGMA), (sg.MEAN, sg.WINSORIZED),
                                              (sg.MEAN, sg.PERCENTILE), (sg.MEAN, sg.SIGMEDIAN),
                                              (sg.MEDIAN, sg.NO_REJEC)])
@pytest.mark.parametrize("normalize", [sg.ADDITIVE_SCALING, sg.ADDITIVE, sg.MULTIPLICATIVE_SCALING,
                                       sg.MULTIPLICATIVE])
def test_fma_load_matches_oracle(gpu_ctx, method, rejection, normalize):
    """realistic coefficients: the check admits the fma load, and the stack equals the oracle"""
    N, H, W = 48, 36, 400
    frames = orc.synth(N, 1, H, W, seed=501 + normalize, maxshift=9)
    sx, sy = orc.synth_shifts(N, seed=501 + normalize, maxshift=9)
    rng = np.random.default_rng(502 + normalize)
    additive = normalize in (sg.ADDITIVE, sg.ADDITIVE_SCALING)
    off = rng.uniform(-80, 80, N) if additive else np.zeros(N)
    mul = np.ones(N) if additive else rng.uniform(0.9, 1.1, N)
    scaled = normalize in (sg.ADDITIVE_SCALING, sg.MULTIPLICATIVE_SCALING)
    scale = 1.0 + rng.uniform(-0.04, 0.04, N) if scaled else np.ones(N)
    off[0], mul[0], scale[0] = 0.0, 1.0, 1.0
    if method == sg.MEDIAN:
        sx = sy = None
    sig = (0.2, 0.1) if rejection == sg.PERCENTILE else (4.0, 3.0)
    desc, keep = sg.make_desc(method, N, W, H, 1, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                              normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert st.path == 1
    want = 2 if normalize == sg.ADDITIVE else 1     # additive with scale 1: the integer offsets
    assert st.norm_fma == want, (st.norm_fma, want)
    if method == sg.MEDIAN:
        rc, ref = orc.stack_median(frames, normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2)
        rej_ref = rej
    else:
        rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=sig, shiftx=sx, shifty=sy,
                                               normalize=normalize, offset=off, mul=mul, scale=scale,
                                               max_thread=2)
    assert rc == 0
    diff = np.argwhere(out != ref)
    assert len(diff) == 0, f"{len(diff)} pixels differ, first {diff[:5].tolist()}"
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
def test_fma_load_refused_keeps_reference(gpu_ctx, rejection):
    """one frame whose coefficients make the fma differ from the reference at one u16 value: the
    check refuses the fma load for the whole call (norm_fma = 0), and the stack, which holds that
    value in the frame, still equals the oracle"""
    s, o, x0, k = _adversarial_frame_coeffs()
    N, H, W = 40, 24, 300
    frames = orc.synth(N, 1, H, W, seed=611, maxshift=6)
    sx, sy = orc.synth_shifts(N, seed=611, maxshift=6)
    rng = np.random.default_rng(612)
    off = np.round(rng.uniform(-60, 60, N) * 2) / 2
    scale = 1.0 + rng.uniform(-0.03, 0.03, N)
    off[0], scale[0] = 0.0, 1.0
    f = 7
    scale[f], off[f] = s, o
    # frame f around x0, so its normalised samples land near k instead of clamping to 0
    frames[f] = np.clip(frames[f].astype(np.int64) - int(frames[f].mean()) + x0, 0, 65535).astype(np.uint16)
    frames[f, 0, H // 2, 10:200] = x0
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=sg.ADDITIVE_SCALING, offset=off, mul=np.ones(N), scale=scale,
                              max_thread=2, max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert st.path == 1
    assert st.norm_fma == 0, "the check admitted an fma load that differs from the reference"
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=sg.ADDITIVE_SCALING, offset=off, mul=np.ones(N),
                                           scale=scale, max_thread=2)
    assert rc == 0
    diff = np.argwhere(out != ref)
    assert len(diff) == 0, f"{len(diff)} pixels differ, first {diff[:5].tolist()}"
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
def test_integer_load_refused_keeps_fma(gpu_ctx, rejection):
    """ADDITIVE (scale 1) with one frame's offset 0.5 + 2^-40: fl(x - 2^-40) rounds back to x for the
    large u16 values, which the integer form (K = 1) cannot reproduce, while the fma rounds the same
    way; the check refuses the integer load, admits the fma (norm_fma = 1), and the stack equals the
    oracle"""
    N, H, W = 40, 24, 300
    frames = orc.synth(N, 1, H, W, seed=621, maxshift=6)
    sx, sy = orc.synth_shifts(N, seed=621, maxshift=6)
    rng = np.random.default_rng(622)
    off = rng.uniform(-60, 60, N)
    off[0] = 0.0
    off[5] = 0.5 + 2.0 ** -40
    frames[5, 0, H // 2, 20:220] = 50000
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=sg.ADDITIVE, offset=off, mul=np.ones(N), scale=np.ones(N),
                              max_thread=2, max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert st.path == 1
    assert st.norm_fma == 1, st.norm_fma
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=sg.ADDITIVE, offset=off, mul=np.ones(N), scale=np.ones(N),
                                           max_thread=2)
    assert rc == 0
    diff = np.argwhere(out != ref)
    assert len(diff) == 0, f"{len(diff)} pixels differ, first {diff[:5].tolist()}"
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


def test_integer_refusal_premise():
    """the refusal case above: at x = 50000 the reference's fl(x - c) (c = offset - 0.5 = 2^-40) is
    x, an integer, so round_to_WORD gives x, while x - ceil(c) = x - 1"""
    c = 2.0 ** -40
    x = 50000.0
    assert (x - c) == x
    y = x - (c + 0.5)
    assert int(y + 0.5) == 50000


@pytest.mark.gpu
@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("normalize", [sg.ADDITIVE_SCALING, sg.MULTIPLICATIVE_SCALING])
def test_captured_samples_near_the_band(gpu_ctx, rejection, normalize):
    """normalised stacks whose columns hold 1..4 out-of-band samples just outside the 256-bin band
    (60..260 ADU beyond it on either side, where the clipping thresholds of the first passes land)
    and some 0 / 65535: the SIGMA / WINSORIZED finishes take the captured values as known samples,
    or find a query among them undecidable and compact the column; every pixel and the counters
    equal the oracle"""
    N, H, W = 96, 40, 256
    rng = np.random.default_rng(700 + 10 * rejection + normalize)
    frames = np.clip(np.rint(2000 + rng.normal(0, 30, (N, 1, H, W))), 0, 65535).astype(np.uint16)
    for y in range(H):
        for x in range(W):
            k = (x + 3 * y) % 5          # 0..4 outliers in this column
            fr = rng.choice(N, size=k, replace=False)
            side = rng.choice([-1, 1], size=k)
            frames[fr, 0, y, x] = np.clip(2000 + side * rng.integers(190, 390, size=k), 1, 65534)
    frames[rng.integers(0, N, 200), 0, rng.integers(0, H, 200), rng.integers(0, W, 200)] = 65535
    frames[rng.integers(0, N, 60), 0, rng.integers(0, H, 60), rng.integers(0, W, 60)] = 0
    loc = 2000 + rng.random(N) * 20
    loc[0] = 2000.0
    scl = 30 + rng.random(N) * 0.6
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), normalize=normalize,
                              offset=off, mul=mul, scale=scale, max_thread=2, max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert st.path == 1
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), normalize=normalize, offset=off,
                                           mul=mul, scale=scale, max_thread=2)
    assert rc == 0
    diff = np.argwhere(out != ref)
    assert len(diff) == 0, f"{len(diff)} pixels differ, first {diff[:5].tolist()}"
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    # most columns hold captured samples; the finish decided most of them
    assert st.compact_pixels < 0.5 * H * W, st.compact_pixels
    print(f"compact {st.compact_pixels} redo {st.chain_pixels} of {H * W}")
