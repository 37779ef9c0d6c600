"""Per-frame normalisation statistics: the device IKSS location / scale
(sg_frame_stats_ikss_device) against the oracle's restatement of statistics() (bit for
bit), and compute_normalization through the C ABI against the oracle (CPU)."""
import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg


@pytest.mark.parametrize("mode", [sg.ADDITIVE, sg.MULTIPLICATIVE, sg.ADDITIVE_SCALING, sg.MULTIPLICATIVE_SCALING])
def test_compute_normalization_matches_oracle(mode):
    rng = np.random.default_rng(mode)
    loc = 1000 + rng.random(9) * 50
    scl = 30 + rng.random(9) * 5
    for ref in (0, 4):
        want = orc.compute_normalization(mode, loc, scl, ref_image=ref)
        got = sg.compute_normalization(mode, loc, scl, ref_image=ref)
        for a, b in zip(got, want):
            assert np.array_equal(a, b)


def _frames():
    rng = np.random.default_rng(7)
    fr = []
    # synthetic star field with shifts / zeros / cosmics (sg_synth), 3 layers
    fr.append(orc.synth(1, 3, 96, 130, seed=5, maxshift=4)[0])
    fr.append(orc.synth(1, 3, 96, 130, seed=6, maxshift=4)[0])
    # 8-bit data (normalised by 255, utils.c:454-459), with zeros (null pixels)
    g = rng.normal(100, 12, size=(3, 96, 130)).clip(0, 255).astype(np.uint16)
    g[0, :5, :] = 0
    fr.append(g)
    # wide 16-bit distribution with outliers
    h = rng.normal(20000, 900, size=(3, 96, 130)).clip(0, 65535).astype(np.uint16)
    h[0, 10:12, :] = 65535
    fr.append(h)
    # nearly constant frame (mad == 0 / sigma == 0 exits)
    c = np.full((3, 96, 130), 777, dtype=np.uint16)
    c[0, 0, :7] = 778
    fr.append(c)
    return np.stack(fr)


@pytest.mark.gpu
def test_ikss_matches_oracle(gpu_ctx):
    import torch
    frames = _frames()
    N, C, H, W = frames.shape
    d = torch.from_numpy(frames.view(np.int16).reshape(-1).copy()).cuda()
    torch.cuda.synchronize()
    rc, loc, scl = gpu_ctx.frame_stats_ikss(d.data_ptr(), N, C, H, W)
    assert rc == 0, gpu_ctx.error()
    for i in range(N):
        orc_rc, l, s = orc.statistics_ikss(frames[i])
        assert orc_rc == 0
        assert loc[i] == l and scl[i] == s, (i, loc[i], l, scl[i], s)


@pytest.mark.gpu
def test_ikss_empty_frame_fails(gpu_ctx):
    import torch
    frames = np.zeros((2, 1, 16, 16), dtype=np.uint16)
    frames[1, 0, 3, 3] = 9
    d = torch.from_numpy(frames.view(np.int16).reshape(-1).copy()).cuda()
    torch.cuda.synchronize()
    rc, loc, scl = gpu_ctx.frame_stats_ikss(d.data_ptr(), 2, 1, 16, 16)
    assert rc != 0
    assert orc.statistics_ikss(frames[0])[0] != 0
    assert (loc[1], scl[1]) == orc.statistics_ikss(frames[1])[1:]
