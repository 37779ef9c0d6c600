"""Perspective warp (a17, sg_warp.hip) vs the numpy restatement of OpenCV's warpPerspective
(tests/warp_ref.py) and hand-derived known answers (identity, integer translations).
Parity with a real OpenCV build is unpinned (OpenCV absent, version unpinned)."""
import numpy as np
import pytest

import sirilgpu as sg
import warp_ref


def _img(C, H, W, seed):
    rng = np.random.default_rng(seed)
    img = (1000 + rng.integers(0, 3000, size=(C, H, W))).astype(np.uint16)
    img[:, H // 3, W // 4] = 65535
    return img


def test_reference_known_answers():
    img = _img(1, 9, 11, 1)
    for interp in (0, 1, 3, 4):
        assert np.array_equal(warp_ref.warp(img, np.eye(3), interp=interp), img)
    # display-coordinate translation by (+2, +1): out(x, y) = in(x - 2, y - 1), 0 outside
    Hm = np.array([[1, 0, 2], [0, 1, 1], [0, 0, 1]], dtype=np.float64)
    disp = img[:, ::-1, :]
    exp = np.zeros_like(disp)
    exp[:, 1:, 2:] = disp[:, :-1, :-2]
    for interp in (0, 1, 3, 4):
        assert np.array_equal(warp_ref.warp(img, Hm, interp=interp), exp[:, ::-1, :]), interp


@pytest.mark.gpu
@pytest.mark.parametrize("interp", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("C", [1, 3])
def test_warp_matches_reference(gpu_ctx, interp, C):
    rng = np.random.default_rng(10 + interp + C)
    H, W = 57, 83
    img = _img(C, H, W, interp)
    for k in range(3):
        a = rng.normal(0, 0.05)
        Hm = np.array([[np.cos(a), -np.sin(a), rng.normal(0, 4)],
                       [np.sin(a), np.cos(a), rng.normal(0, 4)],
                       [rng.normal(0, 2e-4), rng.normal(0, 2e-4), 1.0]])
        out_size = (W, H) if k < 2 else (W + 9, H - 5)
        got = gpu_ctx.warp(img, Hm, out_size, interp)
        exp = warp_ref.warp(img, Hm, out_size, interp)
        assert np.array_equal(got, exp), (interp, C, k, np.argwhere(got != exp)[:5])


@pytest.mark.gpu
def test_warp_identity_and_translation(gpu_ctx):
    img = _img(3, 40, 70, 3)
    Hm = np.array([[1, 0, -3], [0, 1, 5], [0, 0, 1]], dtype=np.float64)
    for interp in (0, 1, 3, 4):
        assert np.array_equal(gpu_ctx.warp(img, np.eye(3), None, interp), img)
        assert np.array_equal(gpu_ctx.warp(img, Hm, None, interp), warp_ref.warp(img, Hm, None, interp))
