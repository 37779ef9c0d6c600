"""Edge cases of the pixel-pair reduce kernel (k_stack_reduce2: SUM / MAX / MIN / MEAN
NO_REJEC, src/stacking/stacking.c:196-355, 824-1128, 1786-1794) and of the half-spectrum
registration passes (register_shift_dft, src/registration/registration.c:182-400).

Reduce: odd and tiny widths, shifts that move one pixel of a lane's pair out of the image
(nx = -1, nx + 1 = W), shifts larger than the image, rows shifted out of the frame, source
pixel 0 (`ii > 0`, :307), normalisation of y-shifted zero rows; each case is compared with
the oracle and with the one-pixel-per-lane kernel (SG_REDUCE1=1), bit for bit.

Registration: the smallest sides (S = 8, 16: the staged small-FFT path and strips that
span a whole half spectrum), odd frame counts (a pair with an empty imaginary part), the
the pass families (fp32 half spectra, fp64 half spectra SG_REG_FP=64, the generic mixed-radix
passes SG_REG_PATH=3) agreeing exactly, and at full size (S = 2048, where
the plain-DFT oracle is too slow) circular shifts recovered exactly with the sign
convention the oracle shows at S = 64.
"""
import os

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg
from test_gpu_stack import assert_same, gpu_stack

pytestmark = pytest.mark.gpu


def _with_env(name, value, fn):
    """fn(ctx) on a context created while the knob is set (knobs are read at sg_init)"""
    old = os.environ.get(name)
    os.environ[name] = value
    try:
        with sg.Context() as ctx:
            return fn(ctx)
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old


EDGE_SHIFTS = [
    ([0, 1, -1, 3, -3], [0, 0, 1, -1, 2]),               # odd x shifts: pairs straddle both edges
    ([0, 40, -40, 7, -8], [0, 3, -2, 9, -9]),            # |sx| >= W for the narrow images
    ([0, 2, -2, 1, -1], [0, 30, -30, 1, 0]),             # rows shifted out of the frame
]


@pytest.mark.parametrize("W", [2, 3, 9, 33, 130])
@pytest.mark.parametrize("case", range(len(EDGE_SHIFTS)))
@pytest.mark.parametrize("method", [sg.SUM, sg.MAX, sg.MIN])
def test_reduce_pairs_edges_sum_max_min(gpu_ctx, W, case, method):
    H, C = 12, 1
    sx, sy = (np.array(a, dtype=np.int32) for a in EDGE_SHIFTS[case])
    N = len(sx)
    rng = np.random.default_rng(1000 * W + 10 * case + method)
    frames = rng.integers(1, 60000, size=(N, C, H, W)).astype(np.uint16)
    if method == sg.SUM:
        rc, ref, mref = orc.stack_sum(frames, sx, sy)
    else:
        rc, ref = orc.stack_maxmin(frames, method == sg.MAX, sx, sy)
    out, _, maxim = gpu_stack(gpu_ctx, frames, method, shiftx=sx, shifty=sy)
    assert_same(out, ref, f"pairs W={W} case={case} method={method}")
    out1, _, maxim1 = _with_env("SG_REDUCE1", "1",
                                lambda c: gpu_stack(c, frames, method, shiftx=sx, shifty=sy))
    assert_same(out, out1, "pairs vs one pixel per lane")
    if method == sg.SUM:
        assert maxim == mref == maxim1


@pytest.mark.parametrize("W", [3, 9, 130])
@pytest.mark.parametrize("normalize", [sg.NO_NORM, sg.ADDITIVE, sg.MULTIPLICATIVE_SCALING])
def test_reduce_pairs_edges_mean(gpu_ctx, W, normalize):
    # |shifty| below the reference's block height (the block offset of stacking.c:1560 is
    # only defined there; the oracle returns -4 otherwise): |shifty| <= 3
    H, C, N = 40, 3, 6
    sx = np.array([0, 1, -1, 5, -140, 2], dtype=np.int32)
    sy = np.array([0, 0, 3, -2, 3, -3], dtype=np.int32)
    rng = np.random.default_rng(77 + W + normalize)
    frames = rng.integers(0, 65535, size=(N, C, H, W)).astype(np.uint16)
    kw = {}
    if normalize != sg.NO_NORM:
        kw = dict(normalize=normalize, offset=rng.uniform(-300, 300, N), mul=rng.uniform(0.8, 1.2, N),
                  scale=rng.uniform(0.9, 1.1, N))
    rc, ref, _ = orc.stack_rejection(frames, sg.NO_REJEC, shiftx=sx, shifty=sy, **kw)
    assert rc == 0
    out, _, _ = gpu_stack(gpu_ctx, frames, sg.MEAN, rejection=sg.NO_REJEC, shiftx=sx, shifty=sy, **kw)
    assert_same(out, ref, f"mean pairs W={W} norm={normalize}")


@pytest.mark.parametrize("S,n", [(8, 2), (8, 3), (16, 4), (16, 7), (32, 3)])
def test_register_small_sides(gpu_ctx, S, n):
    sel = orc.synth(n, 1, S, S, seed=5 * S + n, maxshift=2)[:, 0].copy()
    sel[:, S // 4:S // 4 + 2, S // 2:S // 2 + 2] = 50000
    gx, gy, gq = gpu_ctx.register_dft(sel)
    rx, ry, rq = orc.register_dft(sel)
    assert np.array_equal(gx, rx) and np.array_equal(gy, ry), (gx, rx, gy, ry)


@pytest.mark.parametrize("S,n", [(64, 5), (512, 9)])
def test_register_pass_orders_agree(gpu_ctx, S, n):
    sel = orc.synth(n, 1, S, S, seed=S + 3 * n, maxshift=12)[:, 0].copy()
    res = {"fp32": gpu_ctx.register_dft(sel)}
    res["fp64"] = _with_env("SG_REG_FP", "64", lambda c: c.register_dft(sel))
    res["generic"] = _with_env("SG_REG_PATH", "3", lambda c: c.register_dft(sel))
    for name in ("fp64", "generic"):
        for k in range(3):
            assert np.array_equal(np.nan_to_num(res[name][k], nan=-7.0),
                                  np.nan_to_num(res["fp32"][k], nan=-7.0)), (name, k)


def _scene(S, seed):
    rng = np.random.default_rng(seed)
    scene = rng.integers(0, 3000, size=(S, S)).astype(np.float64)
    scene = (scene + np.roll(scene, 1, 0) + np.roll(scene, 1, 1)) / 3
    scene[S // 3:S // 3 + 5, S // 5:S // 5 + 5] += 30000
    return scene


def _roll_shifts(S, rolls):
    sc = _scene(S, 3)
    return np.stack([np.roll(sc, (dy, dx), axis=(0, 1)) for dx, dy in rolls]).astype(np.uint16)


def _wrap(v, S):
    v = v % S
    return v - S if v > S // 2 else v


def test_register_full_size_known_shifts(gpu_ctx):
    # sign convention of (shiftx, shifty) for a circular roll (dx, dy), from the oracle
    small = [(0, 0), (3, -5)]
    rx, ry, _ = orc.register_dft(_roll_shifts(64, small))
    kx, ky = int(rx[1]) // 3, int(ry[1]) // -5
    assert abs(kx) == 1 and abs(ky) == 1 and rx[1] == 3 * kx and ry[1] == -5 * ky
    S = 2048
    rolls = [(0, 0), (17, -9), (-300, 411), (1023, 0), (0, -1024), (-1, 1), (640, -640)]
    gx, gy, _ = gpu_ctx.register_dft(_roll_shifts(S, rolls))
    for f, (dx, dy) in enumerate(rolls):
        assert gx[f] == _wrap(kx * dx, S) and gy[f] == _wrap(ky * dy, S), (f, gx[f], gy[f], dx, dy)
