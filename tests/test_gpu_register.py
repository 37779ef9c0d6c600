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


def test_register_rejects_non_power_of_two(gpu_ctx):
    sel = np.zeros((2, 48, 48), dtype=np.uint16)
    with pytest.raises(RuntimeError):
        gpu_ctx.register_dft(sel)


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
