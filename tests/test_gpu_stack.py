"""GPU parity of every stacker against the CPU oracle, through the C ABI.

Bit-exact for every output pixel and the rejection counters (integer/median paths and the
mean/sigma-clip paths alike: the kernels replay the reference's decisions exactly).
"""
import os

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg

pytestmark = pytest.mark.gpu

REJ = {sg.PERCENTILE: (0.2, 0.1), sg.SIGMA: (4.0, 3.0), sg.SIGMEDIAN: (4.0, 3.0),
       sg.WINSORIZED: (4.0, 3.0), sg.LINEARFIT: (5.0, 5.0), sg.NO_REJEC: (4.0, 3.0)}


def gpu_stack(ctx, frames, method, rejection=sg.NO_REJEC, sig=(4.0, 3.0), shiftx=None, shifty=None,
              normalize=sg.NO_NORM, offset=None, mul=None, scale=None, max_thread=8, max_rows=0):
    N, C, H, W = frames.shape
    desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, normalize=normalize, sig=sig,
                              shiftx=shiftx, shifty=shifty, offset=offset, mul=mul, scale=scale,
                              max_thread=max_thread, max_number_of_rows=max_rows or H)
    rc, out, rej, maxim = ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, ctx.error()
    return out, rej, maxim


def assert_same(a, b, what):
    if not np.array_equal(a, b):
        idx = np.argwhere(a != b)
        raise AssertionError(f"{what}: {len(idx)} pixels differ, first {idx[:5].tolist()} "
                             f"gpu={a[tuple(idx[0])]} ref={b[tuple(idx[0])]}")


@pytest.mark.parametrize("C", [1, 3])
@pytest.mark.parametrize("rejection", [sg.NO_REJEC, sg.PERCENTILE, sg.SIGMA, sg.WINSORIZED,
                                       sg.SIGMEDIAN, sg.LINEARFIT])
def test_rejection_parity(gpu_ctx, rejection, C):
    N, H, W = 24, 40, 150
    frames = orc.synth(N, C, H, W, seed=11 + C, maxshift=8)
    sx, sy = orc.synth_shifts(N, seed=11 + C, maxshift=8)
    sig = REJ[rejection]
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=1)
    assert rc == 0
    out, rej, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, rejection, sig, sx, sy, max_thread=1)
    assert_same(out, ref, f"rejection {rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("N", [2, 3, 4, 7, 16, 64, 200])
@pytest.mark.parametrize("sig", [(4.0, 3.0), (1.0, 1.0), (2.5, 1.2)])
def test_sigmedian_sorted_path(gpu_ctx, N, sig):
    """SIGMEDIAN on the sorted kernel (replacement groups over the sorted window, exact moments,
    the SIGMA band; more than 4 groups or a decision in the band go to the literal kernel): the
    image and the counters equal the oracle, and with the default sigmas the literal kernel
    takes few pixels"""
    H, W = 20, 130
    frames = _outlier_frames(N, H, W, 700 + N)
    rng = np.random.default_rng(N)
    frames[:, :, :, :8] = rng.integers(900, 1100, size=(N, 1, H, 8)).astype(np.uint16)  # noise-only columns
    sx, sy = orc.synth_shifts(N, seed=700 + N, maxshift=3)
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.SIGMEDIAN, sig=sig, shiftx=sx, shifty=sy, max_thread=2)
    assert rc == 0
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMEDIAN, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=2, max_number_of_rows=H, kernel_path=sg.PATH_SORTED)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    assert gpu_ctx.stats().path == 0
    assert_same(out, ref, f"sigmedian N={N} sig={sig}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if sig == (4.0, 3.0) and N >= 16:
        assert gpu_ctx.stats().slow_pixels <= 0.02 * H * W, gpu_ctx.stats().slow_pixels


@pytest.mark.parametrize("N", [16, 33, 200, 512])
@pytest.mark.parametrize("normalize", [sg.NO_NORM, sg.ADDITIVE_SCALING, sg.MULTIPLICATIVE])
@pytest.mark.parametrize("sig", [(4.0, 3.0), (1.0, 1.0), (2.5, 1.2), (0.3, 0.2)])
def test_sigmedian_hist_path(gpu_ctx, N, normalize, sig):
    """SIGMEDIAN on the histogram kernel (k_stack_hist<3>: the window of never-replaced samples
    as a value interval of the column histogram plus up to 4 replacement groups; decisions in the
    rounding band, a fifth group or a never-ending pass go to the redo list): the image and the
    counters equal the oracle, shifts and normalisation included, and the main kernel is the
    histogram one"""
    H, W = 24, 260
    frames = _outlier_frames(N, H, W, 900 + N)
    rng = np.random.default_rng(N + 7)
    frames[:, :, :, :8] = rng.integers(900, 1100, size=(N, 1, H, 8)).astype(np.uint16)
    sx, sy = orc.synth_shifts(N, seed=900 + N, maxshift=4)
    off = mul = sc = None
    if normalize != sg.NO_NORM:
        loc = 1000 + rng.random(N) * 60
        scl = 30 + rng.random(N) * 5
        off, mul, sc = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.SIGMEDIAN, sig=sig, shiftx=sx, shifty=sy, normalize=normalize,
                                           offset=off, mul=mul, scale=sc, max_thread=2)
    assert rc == 0
    out, rej, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, sg.SIGMEDIAN, sig, sx, sy, normalize=normalize, offset=off,
                            mul=mul, scale=sc, max_thread=2)
    assert gpu_ctx.stats().path == 1
    assert_same(out, ref, f"sigmedian hist N={N} norm={normalize} sig={sig}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("N", [5, 9, 16, 64, 200])
@pytest.mark.parametrize("sig", [(5.0, 5.0), (2.0, 2.0), (1.0, 3.0)])
def test_linearfit_sorted_path(gpu_ctx, N, sig):
    """LINEARFIT on the sorted kernel (the literal double recurrences on the lane's sorted LDS
    column, rejected[] bits with the early break's stale entries, in-place removal): image and
    counters equal the oracle; first-pass early breaks go to the literal kernel"""
    H, W = 20, 130
    frames = _outlier_frames(N, H, W, 800 + N)
    sx, sy = orc.synth_shifts(N, seed=800 + N, maxshift=3)
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.LINEARFIT, sig=sig, shiftx=sx, shifty=sy, max_thread=2)
    assert rc == 0
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.LINEARFIT, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=2, max_number_of_rows=H, kernel_path=sg.PATH_SORTED)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    assert gpu_ctx.stats().path == 0
    assert_same(out, ref, f"linearfit N={N} sig={sig}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if sig == (5.0, 5.0) and N >= 64:
        assert gpu_ctx.stats().slow_pixels <= 0.05 * H * W, gpu_ctx.stats().slow_pixels


@pytest.mark.parametrize("N", [16, 100, 512, 700, 1024])
@pytest.mark.parametrize("normalize", [sg.NO_NORM, sg.ADDITIVE_SCALING])
@pytest.mark.parametrize("sig", [(5.0, 5.0), (2.0, 2.0), (1.0, 3.0)])
def test_linearfit_fast_path(gpu_ctx, N, normalize, sig):
    """LINEARFIT on the decision-exact kernel (k_stack_linfit: the fit from exact integer sums,
    every clip decided outside the bound on the reference's recurrence error, the rest through the
    sorted kernel's replay): image and counters equal the oracle, with shifts, normalisation,
    degenerate columns (constant, an exact ramp: sigma 0, the reference's rounding noise decides)
    and heavy rejection (the early break); few pixels leave the fast kernel"""
    H, W = 12, 200
    frames = _outlier_frames(N, H, W, 1300 + N)
    frames[:, 0, :, 3] = 1234                                                   # constant column
    frames[:, 0, :, 5] = (1000 + 7 * np.arange(N))[:, None].astype(np.uint16)   # exact ramp
    rng = np.random.default_rng(N)
    half = rng.random(N) < 0.5
    frames[half, 0, :, 9] = 60000                                               # half the stack hot
    sx, sy = orc.synth_shifts(N, seed=1300 + N, maxshift=3)
    off = mul = sc = None
    if normalize != sg.NO_NORM:
        loc = 1000 + rng.random(N) * 60
        scl = 30 + rng.random(N) * 5
        off, mul, sc = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.LINEARFIT, sig=sig, shiftx=sx, shifty=sy, normalize=normalize,
                                           offset=off, mul=mul, scale=sc, max_thread=2)
    assert rc == 0
    out, rej, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, sg.LINEARFIT, sig, sx, sy, normalize=normalize, offset=off,
                            mul=mul, scale=sc, max_thread=2)
    st = gpu_ctx.stats()
    assert st.path == 1
    assert_same(out, ref, f"linearfit fast N={N} norm={normalize} sig={sig}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if sig == (5.0, 5.0):
        assert st.chain_pixels <= 0.05 * H * W, st.chain_pixels   # the redo list


def test_sigmedian_never_ending_loop_fails(gpu_ctx):
    """the reference's SIGMEDIAN loop has no cap: {990, 0, 0, 1049} with sig = (2.5, 0.7) halves
    its top pair towards {0, 0, 1, 1}, where both 1s are clipped and replaced by
    round_to_WORD(0.5) = 1 forever (stacking.c:1696-1709; Siril hangs).  The call fails with an
    error instead of hanging the GPU (the oracle is not run: it would not return)"""
    N, H, W = 4, 8, 16
    frames = np.full((N, 1, H, W), 1000, dtype=np.uint16)     # (noise of a few ADU at N = 4 can
    frames[:, 0, 3, 5] = [990, 0, 0, 1049]                     # reach the same kind of cycle)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMEDIAN, sig=(2.5, 0.7), max_thread=1,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc != 0
    assert "never ends" in gpu_ctx.error()
    frames[:, 0, 3, 5] = 1000      # the same stack without that pixel succeeds
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()


@pytest.mark.parametrize("N", [2, 3, 4, 5, 6, 7, 8, 9, 12])
@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED, sg.LINEARFIT])
def test_small_n_stale_state(gpu_ctx, N, rejection):
    """early `break` (N - r <= 4) and stale rejected[] carried across pixels (SURVEY a3 iii)"""
    H, W = 24, 70
    rng = np.random.default_rng(100 + N)
    frames = rng.integers(900, 1100, size=(N, 1, H, W)).astype(np.uint16)
    # outliers on both sides so rejections (and early breaks) happen often
    mask = rng.random(frames.shape)
    frames[mask < 0.08] = 65535
    frames[mask > 0.94] = 0
    sig = (1.0, 1.0) if rejection != sg.LINEARFIT else (1.0, 1.0)
    for max_thread in (1, 3):
        rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=sig, max_thread=max_thread)
        assert rc == 0
        out, rej, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, rejection, sig, max_thread=max_thread)
        assert_same(out, ref, f"N={N} rej={rejection} thr={max_thread}")
        assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("C", [1, 3])
def test_median_parity(gpu_ctx, C):
    N, H, W = 20, 33, 130   # even N: (a+b)/2 truncation
    frames = orc.synth(N, C, H, W, seed=5, maxshift=8)
    rc, ref = orc.stack_median(frames)
    out, _, _ = gpu_stack(gpu_ctx, frames, sg.MEDIAN)
    assert_same(out, ref, "median")


@pytest.mark.parametrize("method", [sg.SUM, sg.MAX, sg.MIN])
@pytest.mark.parametrize("C", [1, 3])
def test_sum_max_min_parity(gpu_ctx, method, C):
    N, H, W = 16, 48, 200
    frames = orc.synth(N, C, H, W, seed=7, maxshift=16)
    sx, sy = orc.synth_shifts(N, seed=7, maxshift=16)
    if method == sg.SUM:
        rc, ref, mref = orc.stack_sum(frames, sx, sy)
    else:
        rc, ref = orc.stack_maxmin(frames, method == sg.MAX, sx, sy)
    out, _, maxim = gpu_stack(gpu_ctx, frames, method, shiftx=sx, shifty=sy)
    assert_same(out, ref, f"method {method}")
    assert out[:, 0, 0].tolist() == ref[:, 0, 0].tolist()
    if method == sg.SUM:
        assert maxim == mref


def test_sum_no_scaling(gpu_ctx):
    """maxim <= 65535: ratio == 1.0 branch (:328-330); pixel 0 stays 0 (:307)"""
    frames = np.full((3, 1, 8, 9), 100, dtype=np.uint16)
    rc, ref, mref = orc.stack_sum(frames)
    out, _, maxim = gpu_stack(gpu_ctx, frames, sg.SUM)
    assert_same(out, ref, "sum small")
    assert out[0, 0, 0] == 0 and maxim == mref == 300


@pytest.mark.parametrize("normalize", [sg.ADDITIVE, sg.MULTIPLICATIVE, sg.ADDITIVE_SCALING,
                                       sg.MULTIPLICATIVE_SCALING])
@pytest.mark.parametrize("method", [sg.MEDIAN, sg.MEAN])
def test_normalization(gpu_ctx, normalize, method):
    N, H, W = 12, 20, 90
    frames = orc.synth(N, 1, H, W, seed=21, maxshift=4)
    rng = np.random.default_rng(3)
    loc = 1000 + rng.random(N) * 50
    scl = 30 + rng.random(N) * 5
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    sx, sy = orc.synth_shifts(N, seed=21, maxshift=4)
    if method == sg.MEDIAN:
        rc, ref = orc.stack_median(frames, normalize, off, mul, scale)
        out, _, _ = gpu_stack(gpu_ctx, frames, sg.MEDIAN, normalize=normalize, offset=off, mul=mul, scale=scale)
    else:
        rc, ref, rr = orc.stack_rejection(frames, sg.SIGMA, shiftx=sx, shifty=sy, normalize=normalize,
                                          offset=off, mul=mul, scale=scale, max_thread=1)
        out, rej, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, sg.SIGMA, shiftx=sx, shifty=sy, normalize=normalize,
                                offset=off, mul=mul, scale=scale, max_thread=1)
        assert np.array_equal(rej, rr)
    assert_same(out, ref, f"norm {normalize} method {method}")


def test_constant_and_knife_edges(gpu_ctx):
    """sigma == 0 stacks (Winsorized 0/0 exit) and integer patterns that put thresholds
    exactly on sample values, forcing the literal (fp80) path"""
    N, H, W = 16, 8, 64
    frames = np.full((N, 1, H, W), 1234, dtype=np.uint16)
    pats = [[1000] * 8 + [1010] * 8, [0] * 15 + [65535], list(range(1000, 1016)),
            [5] * 4 + [9] * 4 + [13] * 8]
    for i, p in enumerate(pats):
        frames[:, 0, i, :] = np.array(p, dtype=np.uint16)[:, None]
    for rej in (sg.SIGMA, sg.WINSORIZED, sg.PERCENTILE, sg.SIGMEDIAN, sg.LINEARFIT):
        for sig in ((4.0, 3.0), (1.0, 1.0), (0.5, 0.5), (2.0, 1.5)):
            rc, ref, rr = orc.stack_rejection(frames, rej, sig=sig, max_thread=2)
            out, rj, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, rej, sig, max_thread=2)
            assert_same(out, ref, f"rej {rej} sig {sig}")
            assert np.array_equal(rj, rr)


def _stack_path(ctx, frames, rejection, sig, sx=None, sy=None, path=sg.PATH_AUTO, max_thread=8):
    N, C, H, W = frames.shape
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=max_thread, max_number_of_rows=H, kernel_path=path)
    rc, out, rej, _ = ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, ctx.error()
    return out, rej, ctx.stats()


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("N", [16, 17, 40, 128, 512])
def test_hist_path_matches_oracle_and_sorted(gpu_ctx, N, rejection):
    """histogram SIGMA / WINSORIZED path (sg_stack_hist.hip) == sorted path == oracle, bit
    for bit"""
    # |shifty| < block height (4 blocks of 16 rows): the reference's heap overflow for
    # larger shifts is not reproduced
    H, W = 64, 160
    frames = orc.synth(N, 1, H, W, seed=300 + N, maxshift=10)
    sx, sy = orc.synth_shifts(N, seed=300 + N, maxshift=10)
    out_h, rej_h, st = _stack_path(gpu_ctx, frames, rejection, (4.0, 3.0), sx, sy, max_thread=2)
    out_s, rej_s, _ = _stack_path(gpu_ctx, frames, rejection, (4.0, 3.0), sx, sy, path=sg.PATH_SORTED,
                                  max_thread=2)
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy, max_thread=2)
    assert rc == 0
    assert_same(out_h, ref, f"hist N={N}")
    assert_same(out_s, ref, f"sorted N={N}")
    assert np.array_equal(rej_h, rej_ref) and np.array_equal(rej_s, rej_ref)
    # the fast path must carry almost every pixel (redo list = pixels re-done by the sort);
    # WINSORIZED's small sigma makes the reference's early break (N - r <= 4) common at
    # small N, and those pixels are redone by design
    limit = 0.05 if (rejection == sg.SIGMA or N >= 40) else 0.2
    assert st.chain_pixels <= limit * H * W, st.chain_pixels


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("normalize", [sg.ADDITIVE, sg.MULTIPLICATIVE, sg.ADDITIVE_SCALING,
                                       sg.MULTIPLICATIVE_SCALING])
def test_hist_path_normalization(gpu_ctx, normalize, rejection):
    """normalised stacks on the histogram path (samples normalised at load, :1635-1652):
    rows shifted out of the frame are normalised zeros, columns shifted out of the image
    stay 0; both interior and image-edge tiles"""
    N, H, W = 40, 64, 300
    frames = orc.synth(N, 1, H, W, seed=410 + normalize, maxshift=10)
    sx, sy = orc.synth_shifts(N, seed=410 + normalize, maxshift=10)
    rng = np.random.default_rng(normalize)
    loc = 1000 + rng.random(N) * 80
    # scale spread of a few %: MULTIPLICATIVE_SCALING puts frame i's background at
    # loc0 * s0 / s_i (:108-119), so a wide spread scatters the frames outside the 256-bin band
    scl = 30 + rng.random(N) * 0.9
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert st.path == 1, "normalised SIGMA / WINSORIZED must take the histogram path"
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2)
    assert rc == 0
    assert_same(out, ref, f"hist norm={normalize} rej={rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    # rows within max|shifty| of the frame border hold normalised zeros of the rows shifted
    # out (round(-offset) etc.): out-of-band values other than 0 / 65535, redone by design
    border = int(np.max(np.abs(sy)))
    assert st.chain_pixels <= (2 * border + 0.05 * H) * W, st.chain_pixels


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("normalize", [sg.ADDITIVE, sg.MULTIPLICATIVE, sg.ADDITIVE_SCALING,
                                       sg.MULTIPLICATIVE_SCALING])
def test_hist_path_normalised_saturation(gpu_ctx, normalize, rejection):
    """normalised samples above 65535 saturate (round_to_WORD, :1635-1652): a bright block near
    65000 with offsets below the reference's (additive) or multipliers above 1
    (multiplicative) sends part of it past 65535 in the histogram path's normalising load"""
    N, H, W = 40, 48, 300
    frames = orc.synth(N, 1, H, W, seed=520 + normalize, maxshift=6)
    rng = np.random.default_rng(520 + normalize)
    frames[:, :, 8:36, 90:170] = (64800 + rng.integers(0, 736, (N, 1, 28, 80))).astype(np.uint16)
    sx, sy = orc.synth_shifts(N, seed=520 + normalize, maxshift=6)
    loc = 1000 - rng.random(N) * 300
    loc[0] = 1000.0
    scl = 30 + rng.random(N) * 0.9
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    assert gpu_ctx.stats().path == 1
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2)
    assert rc == 0
    assert_same(out, ref, f"saturation norm={normalize} rej={rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    # some normalised samples of the block do exceed 65535 (before round_to_WORD's clamp)
    blk = frames[:, 0, 8:36, 90:170].astype(np.float64)
    nv = blk * scale[:, None, None] - off[:, None, None] if normalize in (sg.ADDITIVE, sg.ADDITIVE_SCALING) \
        else blk * scale[:, None, None] * mul[:, None, None]
    assert (nv > 65535.5).any()


def _outlier_frames(N, H, W, seed):
    """synthetic frames with sparse out-of-band samples: 1..6 frames of ~4 % of the pixels hold a
    cosmic ray (20000..65000) or a cold value (1..300), so some pixels keep all their unknown
    values within the histogram kernel's capture (<= 4) and others overflow it"""
    frames = orc.synth(N, 1, H, W, seed=seed, maxshift=6)
    rng = np.random.default_rng(seed)
    npx = int(0.04 * H * W)
    ys, xs = rng.integers(0, H, npx), rng.integers(0, W, npx)
    for y, x in zip(ys, xs):
        k = min(int(rng.integers(1, 7)), N)
        fs = rng.choice(N, k, replace=False)
        hot = rng.random(k) < 0.7
        frames[fs, 0, y, x] = np.where(hot, rng.integers(20000, 65001, k), rng.integers(1, 301, k)).astype(np.uint16)
    return frames


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("normalize", [sg.MULTIPLICATIVE_SCALING, sg.ADDITIVE_SCALING, sg.MULTIPLICATIVE])
@pytest.mark.parametrize("cap", [None, 40])
def test_hist_path_normalised_compact_redo(gpu_ctx, normalize, rejection, cap):
    """normalised stacks: a pixel whose out-of-band samples (besides 0 / 65535) are few leaves
    its sorted column from the histogram kernel (sgh_compact) and the sorted kernel stages it
    without a gather (only when the finish, which takes the captured samples as known values,
    cannot decide the pixel); more than 4 such samples, or a full compact list (cap = 40
    pixels, or half of what the input compacts), send the pixel to the gathering redo list.  All
    must equal the oracle"""
    N, H, W = 64, 48, 300
    seed = 900 + normalize
    frames = _outlier_frames(N, H, W, seed)
    sx, sy = orc.synth_shifts(N, seed=seed, maxshift=6)
    rng = np.random.default_rng(seed + 1)
    loc = 1000 + rng.random(N) * 40
    loc[0] = 1000.0
    scl = 30 + rng.random(N) * 0.9
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2,
                              max_number_of_rows=H)

    def run(ctx):
        rc, out, rej, _ = ctx.stack_host(desc, np.ascontiguousarray(frames))
        assert rc == 0, ctx.error()
        return out, rej, ctx.stats()

    out, rej, st = run(gpu_ctx)
    n0 = int(st.compact_pixels)
    if cap is not None:
        # the SIGMA / WINSORIZED finishes decide most captured pixels themselves since round 6 (CAP), so
        # the compact list is shorter: cap it at half of what this input sends, to reach the overflow
        cap = min(cap, n0 // 2)
        assert cap >= 1, n0
        import os
        old = os.environ.get("SG_HIST_COMPACT")
        os.environ["SG_HIST_COMPACT"] = str(max(cap, 2))
        try:
            with sg.Context() as ctx:
                out, rej, st = run(ctx)
        finally:
            if old is None:
                del os.environ["SG_HIST_COMPACT"]
            else:
                os.environ["SG_HIST_COMPACT"] = old
    assert st.path == 1
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2)
    assert rc == 0
    assert_same(out, ref, f"compact norm={normalize} rej={rejection} cap={cap}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if cap is None:
        # the finish decides most captured pixels; those it cannot still leave as compact columns
        assert st.compact_pixels >= 1, st.compact_pixels
    else:
        assert st.compact_pixels == max(cap, 2), st.compact_pixels


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("tiny", [False, True])
def test_hist_path_additive_fold(gpu_ctx, rejection, tiny):
    """additive normalisation with every offset - 0.5 exact takes the folded kernel (NORM 3);
    one offset of 1e-30 (offset - 0.5 inexact) sends the whole stack to the unfolded one
    (NORM 1); both must equal the oracle.  Offsets include half-integers, where
    round_to_WORD's + 0.5 lands exactly on integers."""
    N, H, W = 36, 40, 300
    frames = orc.synth(N, 1, H, W, seed=77, maxshift=8)
    sx, sy = orc.synth_shifts(N, seed=77, maxshift=8)
    rng = np.random.default_rng(78)
    off = np.round(rng.uniform(-60, 60, N) * 2) / 2          # half-integers
    off[1::3] += rng.uniform(-0.01, 0.01, len(off[1::3]))
    if tiny:
        off[5] = 1e-30
    scale = 1.0 + rng.uniform(-0.03, 0.03, N)
    scale[0] = 1.0
    mul = np.ones(N)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=sg.ADDITIVE_SCALING, offset=off, mul=mul, scale=scale, max_thread=2,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    assert gpu_ctx.stats().path == 1
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=sg.ADDITIVE_SCALING, offset=off, mul=mul, scale=scale,
                                           max_thread=2)
    assert rc == 0
    assert_same(out, ref, f"additive fold tiny={tiny} rej={rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("shifts", [True, False])
@pytest.mark.parametrize("W", [700, 1024])
def test_hist_path_interior_tiles(gpu_ctx, W, shifts):
    """wide frames: interior 128-pixel tiles take the dword-load path (no column checks),
    the two image-edge tile columns the per-pixel path; both must agree with the oracle"""
    N, H = 40, 48
    frames = orc.synth(N, 1, H, W, seed=900 + W, maxshift=12)
    sx, sy = orc.synth_shifts(N, seed=900 + W, maxshift=12) if shifts else (None, None)
    out_h, rej_h, st = _stack_path(gpu_ctx, frames, sg.SIGMA, (3.0, 3.0), sx, sy, max_thread=2)
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.SIGMA, sig=(3.0, 3.0), shiftx=sx, shifty=sy, max_thread=2)
    assert rc == 0
    assert_same(out_h, ref, f"hist W={W} shifts={shifts}")
    assert np.array_equal(rej_h, rej_ref)
    assert st.chain_pixels <= 0.05 * H * W, st.chain_pixels


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("case", ["constant", "uniform", "bimodal", "saturated", "tight_sig", "dark"])
def test_hist_path_adversarial(gpu_ctx, case, rejection):
    """inputs that defeat the histogram's assumptions must fall back, not differ:
    u8 bin overflow (>255 equal samples), tail overflow, medians outside the band,
    decisions on knife edges"""
    N, H, W = 300, 6, 128
    rng = np.random.default_rng(7)
    if case == "constant":
        frames = np.full((N, 1, H, W), 4321, dtype=np.uint16)
        frames[:5, :, ::2, :] = 4400
    elif case == "uniform":
        frames = rng.integers(0, 65536, size=(N, 1, H, W)).astype(np.uint16)
    elif case == "bimodal":
        frames = np.where(rng.random((N, 1, H, W)) < 0.5, 1000, 3000).astype(np.uint16)
        frames += rng.integers(0, 20, size=frames.shape).astype(np.uint16)
    elif case == "saturated":
        frames = np.full((N, 1, H, W), 65535, dtype=np.uint16)
        frames[: N // 3] = rng.integers(60000, 65536, size=(N // 3, 1, H, W)).astype(np.uint16)
    elif case == "tight_sig":
        frames = (1000 + rng.integers(0, 8, size=(N, 1, H, W))).astype(np.uint16)
    else:
        frames = rng.integers(0, 40, size=(N, 1, H, W)).astype(np.uint16)
    sig = (1.0, 0.5) if case == "tight_sig" else (4.0, 3.0)
    out_h, rej_h, _ = _stack_path(gpu_ctx, frames, rejection, sig)
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=sig, max_thread=8)
    assert_same(out_h, ref, case)
    assert np.array_equal(rej_h, rej_ref), (rej_h, rej_ref)


@pytest.mark.parametrize("rejection,sig", [(sg.WINSORIZED, (4.0, 3.0)), (sg.WINSORIZED, (2.0, 1.5)),
                                           (sg.SIGMA, (1.0, 1.0)), (sg.SIGMA, (2.0, 0.8))])
def test_early_break_replay(gpu_ctx, rejection, sig):
    """columns half filled by the shift zero fill (image edges, large shifts) and tight
    sigmas make the reference's `if (N - r <= 4) break;` fire in later passes, leaving this
    pixel's stale rejected[] entries in play: the exact wave replay (k_stack_replay) must
    reproduce the oracle bit for bit, rejection counters included"""
    N, C, H, W = 48, 1, 72, 64     # |shifty| < block height (H/4): the reference's :1560 overflow
    frames = orc.synth(N, C, H, W, seed=4242 + rejection, maxshift=12)
    sx, sy = orc.synth_shifts(N, seed=4242 + rejection, maxshift=12)
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=2)
    assert rc == 0
    out, rej, st = _stack_path(gpu_ctx, frames, rejection, sig, sx, sy, path=sg.PATH_SORTED, max_thread=2)
    assert_same(out, ref, f"rej {rejection} sig {sig}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("dark", [False, True])
@pytest.mark.parametrize("normalize", [sg.ADDITIVE, sg.ADDITIVE_SCALING])
def test_hist_path_border_normalised_zeros(gpu_ctx, normalize, dark, rejection):
    """SIGMA / WINSORIZED (round 6) with additive normalisation: rows whose shifted source row
    leaves a frame hold that frame's normalised zero round_to_WORD(-offset) (zero fill
    :1550-1577, then :1635-1652); the histogram path takes them from the host's border-row table
    instead of the redo list.  dark: background near the normalised zeros, so they fall inside
    the band (the table must step aside and the rows go to the redo list)"""
    N, H, W = 64, 48, 1024
    rng = np.random.default_rng(5 + normalize + 7 * dark)
    loc = (120.0 if dark else 1000.0) + rng.random(N) * 90
    loc[0] = loc.max() + 5     # reference frame brightest: most offsets negative, round(-offset) > 0
    scl = 30 + rng.random(N) * 0.9
    # plain noise around each frame's location (no stars: their out-of-band samples would send
    # pixels to the redo list for reasons of their own), 0.05 % cosmics at 65535
    frames = np.clip(rng.normal(loc[:, None, None, None], 20.0, (N, 1, H, W)), 0, 65535).astype(np.uint16)
    frames[rng.random(frames.shape) < 5e-4] = 65535
    sx, sy = orc.synth_shifts(N, seed=77 + normalize, maxshift=10)
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=3,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert st.path == 1
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=3)
    assert rc == 0
    assert_same(out, ref, f"border zeros norm={normalize} dark={dark} rej={rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if not dark:
        border = int(np.max(np.abs(sy)))
        # without the table every pixel of the 2 x border rows would be redone; now only those of
        # the two image-edge tiles (columns < 128 and >= 896 here) and of the few rows whose
        # thresholds or medians fall among the normalised zeros (measured: 6.7 k of 20.5 k)
        assert st.chain_pixels < border * W, st.chain_pixels


@pytest.mark.parametrize("rejection", [sg.SIGMA, sg.WINSORIZED])
@pytest.mark.parametrize("normalize", [sg.ADDITIVE, sg.ADDITIVE_SCALING])
def test_hist_path_edge_corners_stars(gpu_ctx, normalize, rejection):
    """additive normalisation at the image corners: frames shifted out in BOTH directions (x
    and y, shifts up to 12 in every sign) give the x shift's raw 0 where the y shift alone
    gives the normalised zero (:1628-1632 vs :1550-1577, :1635-1652), image-edge tiles hold
    both kinds in their border rows, and stars (bright Gaussian blobs) sit on the corners and
    the edges so those pixels also carry out-of-band samples of their own"""
    N, H, W = 48, 56, 400
    rng = np.random.default_rng(900 + normalize + 3 * rejection)
    loc = 1000.0 + rng.random(N) * 90
    loc[0] = loc.max() + 5
    scl = 30 + rng.random(N) * 0.9
    yy, xx = np.mgrid[0:H, 0:W]
    scene = np.zeros((H, W))
    for cy, cx in [(2, 3), (H - 3, W - 4), (4, W - 6), (H - 5, 5), (H // 2, 1), (1, W // 2), (H - 2, W // 3)]:
        scene += 20000.0 * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * 2.0 ** 2))
    frames = np.clip(loc[:, None, None, None] + scene[None, None] + rng.normal(0, 20.0, (N, 1, H, W)), 0,
                     65535).astype(np.uint16)
    sx = rng.integers(-12, 13, N).astype(np.int32)
    sy = rng.integers(-12, 13, N).astype(np.int32)
    sx[0] = sy[0] = 0
    off, mul, scale = orc.compute_normalization(normalize, loc, scl, ref_image=0)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                              normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, np.ascontiguousarray(frames))
    assert rc == 0, gpu_ctx.error()
    assert gpu_ctx.stats().path == 1
    rc, ref, rej_ref = orc.stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=sx, shifty=sy,
                                           normalize=normalize, offset=off, mul=mul, scale=scale, max_thread=2)
    assert rc == 0
    assert_same(out, ref, f"corners norm={normalize} rej={rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("cap", [None, "4", "12"])
def test_hist_winsorized_iteration_cap(gpu_ctx, cap):
    """pixels whose Winsorize pass needs more inner iterations than SG_WINS_CAP leave the
    histogram path for the wave-per-pixel replay: results and counters stay the oracle's.
    Several 65535s / zeros per pixel make passes of tens to hundreds of iterations."""
    import os
    N, H, W = 256, 8, 256
    rng = np.random.default_rng(2024)
    frames = rng.normal(2000, 30, size=(N, 1, H, W)).round().astype(np.uint16)
    k = rng.integers(0, 9, size=(H, W))                    # 0..8 extreme samples per pixel
    for y in range(H):
        for x in range(W):
            idx = rng.choice(N, size=k[y, x], replace=False)
            frames[idx, 0, y, x] = 65535 if (x + y) % 2 else 0
    old = os.environ.get("SG_WINS_CAP")
    if cap is not None:
        os.environ["SG_WINS_CAP"] = cap
    try:
        with sg.Context() as c:
            out_h, rej_h, st = _stack_path(c, frames, sg.WINSORIZED, (4.0, 3.0))
    finally:
        if old is None:
            os.environ.pop("SG_WINS_CAP", None)
        else:
            os.environ["SG_WINS_CAP"] = old
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.WINSORIZED, sig=(4.0, 3.0), max_thread=8)
    assert rc == 0
    assert_same(out_h, ref, f"cap={cap}")
    assert np.array_equal(rej_h, rej_ref), (rej_h, rej_ref)
    if cap == "4":
        assert st.chain_pixels > 0.2 * H * W, st.chain_pixels   # the cap did send pixels away


def test_block_overflow_shift_refused(gpu_ctx):
    """a shift reaching above a block that does not start at the top of the image: the reference
    reads the block's rows 2 start_row too low and past its buffer (stacking.c:1555-1561, the
    oracle returns -4); the library refuses instead of silently zero filling"""
    N, C, H, W = 8, 1, 24, 64
    frames = orc.synth(N, C, H, W, seed=4, maxshift=2)
    sx = np.zeros(N, np.int32)
    sy = np.zeros(N, np.int32)
    sy[3] = -9                          # 4 threads, 24 rows: blocks of 6 rows; -9 < -6
    rc, ref, _ = orc.stack_rejection(frames, sg.SIGMA, shiftx=sx, shifty=sy, max_thread=4)
    assert rc == -4
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.SIGMA, shiftx=sx, shifty=sy, max_thread=4,
                              max_number_of_rows=H)
    rc, out, rej, _ = gpu_ctx.stack_host(desc, frames)
    assert rc == -1 and "overflows" in gpu_ctx.error()
    # one thread: 4 blocks of 6 rows too (H / rows < 4); with max_number_of_rows 24 and a shift
    # that stays below the first block start it stacks
    sy[3] = -5
    rc, ref, rr = orc.stack_rejection(frames, sg.SIGMA, shiftx=sx, shifty=sy, max_thread=4)
    assert rc == 0
    out, rej, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, sg.SIGMA, shiftx=sx, shifty=sy, max_thread=4)
    assert_same(out, ref, "shift below the block height")


def _export_ctx():
    """a context with SG_WINS_EXPORT=1 (the knob is read when the context opens)"""
    old = os.environ.get("SG_WINS_EXPORT")
    os.environ["SG_WINS_EXPORT"] = "1"
    try:
        return sg.Context([0])
    finally:
        if old is None:
            del os.environ["SG_WINS_EXPORT"]
        else:
            os.environ["SG_WINS_EXPORT"] = old


@pytest.mark.parametrize("N,H,W,M", [(16, 48, 200, 3), (40, 64, 300, 10), (256, 40, 384, 6), (96, 72, 260, 12)])
def test_wins_export_matches_oracle(N, H, W, M):
    """WINSORIZED with the slow columns exported from their tiles and finished by k_hist_slow
    (SG_WINS_EXPORT): image and counters == the oracle and == the in-tile finish.  The synthetic
    frames hold cosmics (65535) and dead pixels (0), and the shifted border rows zeros, so many
    columns are exported; at M = 10 / 12 more than a quarter of the columns are slow and the slot
    pool (a quarter of the pixels) overflows, so the columns beyond it finish in their tiles"""
    frames = orc.synth(N, 1, H, W, seed=900 + N, maxshift=M)
    sx, sy = orc.synth_shifts(N, seed=900 + N, maxshift=M)
    rc, ref, rej_ref = orc.stack_rejection(frames, sg.WINSORIZED, sig=(4.0, 3.0), shiftx=sx, shifty=sy, max_thread=2)
    assert rc == 0
    with _export_ctx() as ctx:
        out_x, rej_x, st = _stack_path(ctx, frames, sg.WINSORIZED, (4.0, 3.0), sx, sy, max_thread=2)
    assert st.exported_pixels > 0, "no column was exported"
    assert st.exported_pixels <= (H * W // 4 + 63) // 64 * 64
    assert_same(out_x, ref, f"exported N={N}")
    assert np.array_equal(rej_x, rej_ref), (rej_x, rej_ref)
