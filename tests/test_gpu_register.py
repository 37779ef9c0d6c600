"""GPU DFT registration (sg_register_dft_u16, replaces register_shift_dft,
src/registration/registration.c:182-400) against the oracle and the golden fixture.

Shifts: bit-exact (integer arg-max of the correlation; inputs chosen with a clear peak, the
FFTW near-tie case is parity-unpinned).  Quality: QualityEstimate is integer
arithmetic followed by the same double operations, so it is compared exactly too.
"""
import os

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _same_q(a, b):
    return np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(a[~np.isnan(a)], b[~np.isnan(b)])


@pytest.mark.parametrize("S", [16, 64, 128, 256])
@pytest.mark.parametrize("n", [2, 5, 8])
def test_register_matches_oracle(gpu_ctx, S, n):
    sel = orc.synth(n, 1, S, S, seed=S + n, maxshift=7)[:, 0].copy()
    # bright structure so the quality map is populated
    sel[:, S // 3:S // 3 + 3, S // 2:S // 2 + 3] = 40000
    gx, gy, gq = gpu_ctx.register_dft(sel)
    rx, ry, rq = orc.register_dft(sel)
    assert np.array_equal(gx, rx) and np.array_equal(gy, ry), (gx, rx, gy, ry)
    assert _same_q(gq, rq), (gq, rq)


def test_register_circular_shift_and_reference(gpu_ctx):
    S = 256
    rng = np.random.default_rng(1)
    scene = rng.integers(0, 3000, size=(S, S)).astype(np.float64)
    scene = (scene + np.roll(scene, 1, 0) + np.roll(scene, 1, 1)) / 3
    shifts = [(0, 0), (9, -4), (-33, 17), (100, 0), (-1, -127), (5, 5), (-64, 64)]
    sel = np.stack([np.roll(scene, (dy, dx), axis=(0, 1)) for dx, dy in shifts]).astype(np.uint16)
    for ref in (0, 3):
        gx, gy, gq = gpu_ctx.register_dft(sel, ref_image=ref)
        rx, ry, rq = orc.register_dft(sel, ref_image=ref)
        assert np.array_equal(gx, rx) and np.array_equal(gy, ry)
        assert gx[ref] == 0 and gy[ref] == 0
        assert _same_q(gq, rq)


def test_register_excluded_frames(gpu_ctx):
    S = 64
    sel = orc.synth(6, 1, S, S, seed=4, maxshift=5)[:, 0].copy()
    inc = np.array([1, 0, 1, 1, 0, 1], dtype=np.int32)
    gx, gy, gq = gpu_ctx.register_dft(sel, included=inc)
    rx, ry, rq = orc.register_dft(sel, included=inc)
    keep = inc.astype(bool)
    assert np.array_equal(gx[keep], rx[keep]) and np.array_equal(gy[keep], ry[keep])
    assert _same_q(gq[keep], rq[keep])


def test_register_golden(gpu_ctx):
    d = np.load(os.path.join(ROOT, "tests", "golden", "register_dft64.npz"), allow_pickle=False)
    gx, gy, gq = gpu_ctx.register_dft(d["sel"])
    assert np.array_equal(gx, d["shiftx"]) and np.array_equal(gy, d["shifty"])
    assert _same_q(gq, d["quality"])


# ---- any selection side (FFTW plans every S, registration.c:251-257) ----

def _numpy_shifts(sel, ref=0):
    """register_shift_dft's arg-max with an independent FFT (numpy pocketfft, float64)"""
    n, S, _ = sel.shape
    R = np.fft.fft2(sel[ref].astype(np.float64))
    sx, sy = np.zeros(n, np.int32), np.zeros(n, np.int32)
    for f in range(n):
        if f == ref:
            continue
        c = np.fft.ifft2(R * np.conj(np.fft.fft2(sel[f].astype(np.float64)))).real
        k = int(np.argmax(c))
        y, x = divmod(k, S)
        sy[f] = y - S if y > S // 2 else y
        sx[f] = x - S if x > S // 2 else x
    return sx, sy


@pytest.mark.parametrize("S", [6, 7, 12, 35, 48, 97, 100, 105, 120])
def test_register_any_side_matches_oracle(gpu_ctx, S):
    """mixed radix (2, 3, 5, 7 factors) and Bluestein (97: prime) against the oracle's
    mixed-radix DFT, shifts and qualities exactly"""
    n = 5
    sel = orc.synth(n, 1, S, S, seed=S + 3, maxshift=min(7, S // 4))[:, 0].copy()
    sel[:, S // 3:S // 3 + 2, S // 2:S // 2 + 2] = 40000
    gx, gy, gq = gpu_ctx.register_dft(sel)
    rx, ry, rq = orc.register_dft(sel)
    assert np.array_equal(gx, rx) and np.array_equal(gy, ry), (S, gx, rx, gy, ry)
    assert _same_q(gq, rq), (gq, rq)


@pytest.mark.parametrize("S", [1500, 2940, 1009, 1234])
def test_register_large_non_power_of_two(gpu_ctx, S):
    """1500 = 2^2 3 5^3 and 2940 = 2^2 3 5 7^2 (mixed radix, in-place LDS passes), 1009 (prime)
    and 1234 = 2 x 617 (Bluestein, m = 4096):
    the arg-max equals an independent numpy FFT's (translations recovered to a pixel);
    qualities equal the oracle's QualityEstimate"""
    n, M = 6, 12
    sel = orc.synth(n, 1, S, S, seed=S, maxshift=M)[:, 0].copy()
    gx, gy, gq = gpu_ctx.register_dft(sel, ref_image=0)
    ex, ey = orc.synth_shifts(n, seed=S, maxshift=M)
    nx, ny = _numpy_shifts(sel)
    assert np.array_equal(gx, nx) and np.array_equal(gy, ny), (gx, nx, gy, ny)
    # the arg-max is the parity target; the synthetic translation itself is only recovered to
    # within a pixel (the scene is not periodic: at S = 1009 two frames' peaks sit one off)
    assert np.abs(gx - ex).max() <= 1 and np.abs(gy - ey).max() <= 1, (gx, ex, gy, ey)
    rq = np.array([orc.quality(sel[f]) for f in range(n)])
    q_min = q_max = rq[0]                   # normalizeQualityData with register_shift_dft's min / max
    for q in rq[1:]:
        q_max = q if q > q_max else q_max
        q_min = q_min if q_min < q else q
    assert _same_q(gq, (rq - q_min) / (q_max - q_min))


def test_register_generic_path_on_power_of_two(gpu_ctx):
    """SG_REG_PATH=3 sends a power-of-two side through the generic passes: same shifts and
    qualities as the fused half-spectrum passes"""
    S, n = 256, 7
    sel = orc.synth(n, 1, S, S, seed=77, maxshift=9)[:, 0].copy()
    gx, gy, gq = gpu_ctx.register_dft(sel)
    os.environ["SG_REG_PATH"] = "3"
    try:
        with sg.Context() as c3:
            hx, hy, hq = c3.register_dft(sel)
    finally:
        del os.environ["SG_REG_PATH"]
    assert np.array_equal(gx, hx) and np.array_equal(gy, hy) and _same_q(gq, hq)


@pytest.mark.parametrize("S", [105, 1500])
def test_register_generic_fused_columns_match_unfused(gpu_ctx, S):
    """the fused generic column pass (k_gen_cols_xpower: rows kx and S - kx of the transposed
    spectrum in one workgroup) gives the three-kernel sequence's shifts and qualities
    (SG_REG_GENFUSE=0)"""
    n = 5
    sel = orc.synth(n, 1, S, S, seed=S + 5, maxshift=min(9, S // 4))[:, 0].copy()
    gx, gy, gq = gpu_ctx.register_dft(sel)
    os.environ["SG_REG_GENFUSE"] = "0"
    try:
        with sg.Context() as c0:
            hx, hy, hq = c0.register_dft(sel)
    finally:
        del os.environ["SG_REG_GENFUSE"]
    assert np.array_equal(gx, hx) and np.array_equal(gy, hy) and _same_q(gq, hq)


def test_register_wave_columns_match_block_columns(gpu_ctx):
    """S = 2048: the wave-level fp32 column pass (k_reg_cols_xpower_w, 32 x 64 four-step
    transforms in registers) gives the block-level pass's shifts and qualities (SG_REG_WCOL=0),
    and the numpy arg-max; an odd frame count exercises the pair with an empty imaginary frame"""
    S, n = 2048, 7
    sel = orc.synth(n, 1, S, S, seed=91, maxshift=14)[:, 0].copy()
    gx, gy, gq = gpu_ctx.register_dft(sel)
    os.environ["SG_REG_WCOL"] = "0"
    try:
        with sg.Context() as c0:
            hx, hy, hq = c0.register_dft(sel)
    finally:
        del os.environ["SG_REG_WCOL"]
    assert np.array_equal(gx, hx) and np.array_equal(gy, hy) and _same_q(gq, hq)
    nx, ny = _numpy_shifts(sel)
    assert np.array_equal(gx, nx) and np.array_equal(gy, ny), (gx, nx, gy, ny)


@pytest.mark.parametrize("S", [256, 2048])
def test_register_fp32_passes_match_fp64(gpu_ctx, S):
    """the fp32 half-spectrum passes (default, SG_REG_FP=32) give the fp64 passes' shifts and
    qualities: a maximum is decided in fp32 only when it beats every other entry by more than
    the fp32 tolerance, otherwise the pair is re-run in fp64"""
    n = 9 if S == 256 else 5
    sel = orc.synth(n, 1, S, S, seed=S + 11, maxshift=12)[:, 0].copy()
    gx, gy, gq = gpu_ctx.register_dft(sel)
    os.environ["SG_REG_FP"] = "64"
    try:
        with sg.Context() as c64:
            hx, hy, hq = c64.register_dft(sel)
    finally:
        del os.environ["SG_REG_FP"]
    assert np.array_equal(gx, hx) and np.array_equal(gy, hy) and _same_q(gq, hq)
    nx, ny = _numpy_shifts(sel)
    assert np.array_equal(gx, nx) and np.array_equal(gy, ny), (gx, nx, gy, ny)


def _periodic_pair(S, dx, dy, seed):
    """ref periodic with period S/2 along x, img = ref circularly translated by (dy, dx):
    the correlation has two exactly equal maxima, at kx and kx + S/2"""
    rng = np.random.default_rng(seed)
    half = rng.integers(500, 3000, size=(S, S // 2)).astype(np.int64)
    ref = np.concatenate([half, half], axis=1)
    img = np.roll(ref, (dy, dx), axis=(0, 1))
    return ref, img


@pytest.mark.parametrize("S", [64, 60])
def test_register_exact_tie_takes_lowest_index(gpu_ctx, S):
    """an exact tie between two correlation maxima is detected (top-2 margin) and decided by
    exact integer correlations: the lowest row-major index wins (FFTW's own choice between
    exactly equal values is unspecified -- parity unpinned)"""
    ref, img = _periodic_pair(S, 3, 5, seed=S)
    sel = np.stack([ref, img]).astype(np.uint16)
    gx, gy, _ = gpu_ctx.register_dft(sel)
    st = gpu_ctx.stats()
    # exact correlations at the two candidates: c(k) = sum_n ref(n + k) img(n)
    k1 = ((-5) % S, (-3) % S)
    k2 = (k1[0], (k1[1] + S // 2) % S)
    e1, e2 = orc.xcorr_at(ref, img, *k1), orc.xcorr_at(ref, img, *k2)
    assert e1 == e2
    lo = min(k1[0] * S + k1[1], k2[0] * S + k2[1])
    y, x = divmod(lo, S)
    assert (gx[1], gy[1]) == (x - S if x > S // 2 else x, y - S if y > S // 2 else y)
    assert st.reg_ties_resolved >= 1
    if S == 64 and os.environ.get("SG_REG_FP", "32") == "32":
        assert st.reg_fp64_reruns >= 1          # the fp32 passes handed the pair to fp64 first


@pytest.mark.gpu
def test_register_tie_rerun_on_fresh_context_large_side():
    """a single fp32 pair re-run in fp64 on a FRESH context at S = 1024: the fp64 plane is twice
    the fp32 pair plane, and the work buffer is sized for it (no other test's larger buffer to
    hide an overflow)"""
    S = 1024
    ref, img = _periodic_pair(S, 3, 5, seed=S)
    sel = np.stack([ref, img]).astype(np.uint16)
    with sg.Context() as c:
        gx, gy, _ = c.register_dft(sel)
        st = c.stats()
    k1 = ((-5) % S, (-3) % S)
    k2 = (k1[0], (k1[1] + S // 2) % S)
    lo = min(k1[0] * S + k1[1], k2[0] * S + k2[1])
    y, x = divmod(lo, S)
    assert (gx[1], gy[1]) == (x - S if x > S // 2 else x, y - S if y > S // 2 else y)
    assert st.reg_ties_resolved >= 1
    if os.environ.get("SG_REG_FP", "32") == "32":
        assert st.reg_fp64_reruns >= 1


def test_register_near_tie_takes_exact_maximum(gpu_ctx):
    """two maxima differing by exactly 1 in the integer correlation (a cross term of two
    single-pixel +1 perturbations, one in each frame, lands on the later one): flagged and
    decided by the exact correlation -> the later index"""
    S, dx, dy = 64, 3, 5
    ref, img = _periodic_pair(S, dx, dy, seed=9)
    k1 = ((-dy) % S, (-dx) % S)
    k2 = (k1[0], (k1[1] + S // 2) % S)
    first, second = sorted([k1, k2], key=lambda k: k[0] * S + k[1])
    n0 = (7, 11)
    m0 = ((n0[0] + second[0]) % S, (n0[1] + second[1]) % S)     # m0 - n0 = the later maximum
    ref = ref.copy()
    img = img.copy()
    ref[m0] += 1
    img[n0] += 1
    ea, eb = orc.xcorr_at(ref, img, *first), orc.xcorr_at(ref, img, *second)
    assert eb - ea == 1
    sel = np.stack([ref, img]).astype(np.uint16)
    gx, gy, _ = gpu_ctx.register_dft(sel)
    y, x = second
    assert (gx[1], gy[1]) == (x - S if x > S // 2 else x, y - S if y > S // 2 else y)
    assert gpu_ctx.stats().reg_ties_resolved >= 1


def test_register_flat_frames_unresolved(gpu_ctx):
    """constant frames: every shift ties; more candidates than the cap, so the FFT arg-max
    stands and both registered frames are reported unresolved"""
    sel = np.full((3, 32, 32), 1234, np.uint16)
    gpu_ctx.register_dft(sel)
    assert gpu_ctx.stats().reg_ties_unresolved == 2


@pytest.mark.parametrize("world,ref", [(2, 0), (3, 5)])
def test_register_raw_shards_reassemble(gpu_ctx, world, ref):
    """sg_register_dft_u16_device_raw on frame shards (frames sharded over GPUs,
    shifts / raw qualities gathered, normalizeQualityData over all frames) equals the
    single-call sg_register_dft_u16 result exactly; shards run one after the other here (the
    gloo test covers the all_gather path)."""
    import torch
    import sirilgpu_dist as sd
    S, n = 128, 9
    sel = orc.synth(n, 1, S, S, seed=99 + world, maxshift=6)[:, 0].copy()
    sel[:, S // 3:S // 3 + 3, S // 2:S // 2 + 3] = 40000
    sel[4, 10:14, 90:94] = 62000
    gx, gy, gq = gpu_ctx.register_dft(sel, ref_image=ref)
    d_sel = torch.from_numpy(sel.view(np.int16)).cuda()
    torch.cuda.synchronize()
    sx = np.zeros(n, np.int32)
    sy = np.zeros(n, np.int32)
    qraw = np.zeros(n, np.float64)
    for r in range(world):
        b, e = sd.frame_band(r, world, n)
        mine = np.zeros(n, np.int32)
        mine[b:e] = 1
        px, py, pq = gpu_ctx.register_dft_device(d_sel.data_ptr(), n, S, ref_image=ref, included=mine,
                                                 raw_quality=True)
        torch.cuda.synchronize()
        sx[b:e], sy[b:e], qraw[b:e] = px[b:e], py[b:e], pq[b:e]
        qraw[ref] = pq[ref]
    sx[ref] = sy[ref] = 0
    q = sd.normalize_quality(qraw, n, ref, None)
    assert np.array_equal(sx, gx) and np.array_equal(sy, gy)
    assert _same_q(q, gq), (q, gq)
    # the raw values are QualityEstimate's (the oracle's, exactly)
    assert _same_q(qraw, np.array([orc.quality(sel[f]) for f in range(n)]))


@pytest.mark.parametrize("S,x0,y0", [(2048, 1976, 976), (64, 7, 3), (60, 12, 5), (64, 8, 2)])
def test_register_pitched_window_matches_extracted(gpu_ctx, S, x0, y0):
    """selections read in place from resident [C][H][W] frames (sg_register_dft_u16_device_pitched:
    layer 1's S x S window at (x0, y0), frame pitch C H W, row pitch W) register exactly as the
    extracted contiguous selections do: shifts and raw / normalised qualities (the wave-level
    S = 2048 rows, the block rows at 64, the generic passes at 60; an odd x0 takes k_quality_sub's
    unaligned loads)"""
    import torch
    N, C = (6, 2) if S == 2048 else (9, 3)
    H, W = S + 2 * y0 + 3, S + x0 + 17
    frames = orc.synth(N, C, H, W, seed=S + x0, maxshift=5)
    if S != 2048:
        frames[:, 1, y0 + 10:y0 + 14, x0 + 20:x0 + 24] = 40000      # structure for QualityEstimate
    d = torch.from_numpy(frames.view(np.int16).reshape(-1)).cuda()
    sel = np.ascontiguousarray(frames[:, 1, y0:y0 + S, x0:x0 + S])
    ds = torch.from_numpy(sel.view(np.int16).reshape(-1)).cuda()
    torch.cuda.synchronize()
    inc = np.ones(N, np.int32)
    inc[2] = 0
    want = gpu_ctx.register_dft_device(ds.data_ptr(), N, S, ref_image=1, included=inc)
    base = d.data_ptr() + 2 * (H * W + y0 * W + x0)
    got = gpu_ctx.register_dft_device(base, N, S, ref_image=1, included=inc, frame_pitch=C * H * W, row_pitch=W)
    for a, b in zip(got, want):
        assert np.array_equal(a, b, equal_nan=True), (a, b)
    raw_w = gpu_ctx.register_dft_device(ds.data_ptr(), N, S, ref_image=1, included=inc, raw_quality=True)[2]
    raw_g = gpu_ctx.register_dft_device(base, N, S, ref_image=1, included=inc, raw_quality=True, frame_pitch=C * H * W,
                                        row_pitch=W)[2]
    assert np.array_equal(raw_g, raw_w, equal_nan=True)
    if S <= 64:
        rx, ry, _ = orc.register_dft(sel, ref_image=1, included=inc)
        m = inc.astype(bool)
        assert np.array_equal(got[0][m], rx[m]) and np.array_equal(got[1][m], ry[m])


def test_register_pitched_tie_exact(gpu_ctx):
    """the exact integer correlations of a near tie (k_reg_exact) read the pitched selections"""
    import torch
    S, pad = 64, 9
    ref, img = _periodic_pair(S, 3, 5, seed=S)
    big = np.zeros((2, S + pad, S + 2 * pad), np.uint16)
    big[:, pad:, pad:pad + S] = np.stack([ref, img]).astype(np.uint16)
    d = torch.from_numpy(big.view(np.int16).reshape(-1)).cuda()
    torch.cuda.synchronize()
    W = S + 2 * pad
    gx, gy, _ = gpu_ctx.register_dft_device(d.data_ptr() + 2 * (pad * W + pad), 2, S, frame_pitch=(S + pad) * W,
                                            row_pitch=W)
    cx, cy, _ = gpu_ctx.register_dft(np.stack([ref, img]).astype(np.uint16))
    assert (gx[1], gy[1]) == (cx[1], cy[1])
    assert gpu_ctx.stats().reg_ties_resolved >= 1


@pytest.mark.parametrize("rpw", [3, 6, 12])
def test_register_quality_fold_matches(gpu_ctx, rpw):
    """SG_REG_QFOLD (default 12): QualityEstimate's 3 x 3 subsample taken inside the wave-level forward
    rows (r consecutive rows per wave) gives k_quality_sub's raw qualities, the oracle's
    QualityEstimate and the same shifts; an odd frame count (a pair with no second frame), an
    excluded frame, a reference that is not frame 0 and a pitched selection window"""
    import torch
    S, N, x0, y0 = 2048, 6, 5, 3
    H, W = S + y0 + 2, S + x0 + 9
    frames = orc.synth(N, 1, H, W, seed=300 + rpw, maxshift=6)[:, 0].copy()
    frames[:, y0 + 700:y0 + 706, x0 + 900:x0 + 906] = 52000      # structure above the threshold
    frames[3, y0 + 1500:y0 + 1503, x0 + 100:x0 + 103] = 65535
    d = torch.from_numpy(frames.view(np.int16).reshape(-1)).cuda()
    torch.cuda.synchronize()
    inc = np.ones(N, np.int32)
    inc[4] = 0
    base = d.data_ptr() + 2 * (y0 * W + x0)
    res = {}
    for r in (0, rpw):
        os.environ["SG_REG_QFOLD"] = str(r)
        try:
            with sg.Context() as c:
                res[r] = (c.register_dft_device(base, N, S, ref_image=2, included=inc, raw_quality=True,
                                                frame_pitch=H * W, row_pitch=W),
                          c.register_dft_device(base, N, S, ref_image=2, included=inc, frame_pitch=H * W, row_pitch=W))
        finally:
            del os.environ["SG_REG_QFOLD"]
    (want, norm_w), (got, norm) = res[0], res[rpw]
    m = inc.astype(bool)
    for a, b in zip(got, want):
        assert np.array_equal(a[m], b[m], equal_nan=True), (a, b)
    assert np.array_equal(norm[2][m], norm_w[2][m], equal_nan=True)
    for f in (2, 3, 5):
        sel = np.ascontiguousarray(frames[f, y0:y0 + S, x0:x0 + S])
        assert _same_q(np.array([got[2][f]]), np.array([orc.quality(sel)])), (f, got[2][f])
