"""Golden registration results for BASELINE configs[1] and configs[4] at their full size
(TEST INFRASTRUCTURE; run here, on the CPU, and commit the .npz it writes).

    python tests/golden/make_golden_fullsize.py

The frames are the synthetic sequence of include/sg_synth.h (the oracle's or_synth_window
generates the registration selection without the rest of the frame).  For every frame the
script follows register_shift_dft (src/registration/registration.c:256-351) with an
independent FFT (numpy's pocketfft in float64, not the oracle's and not the GPU's):
c = IFFT2(FFT2(ref) conj FFT2(img)), shift = first index of the maximum of c (row-major),
values > S/2 wrapped to negative.  The exact integer correlation (oracle or_xcorr_at) is
evaluated at the winner and at the runner-up so that the fixture records that the choice is
not a near tie (FFT rounding cannot move it), and the shifts are checked against the
translations the generator applied.  Quality: the oracle's QualityEstimate restatement
(src/algos/quality.c:46-218), raw per frame (normalizeQualityData is applied by the test).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as orc  # noqa: E402

CONFIGS = {
    # name: (nframes, C, H, W, layer, S, seed, maxshift) -- bench.py main_config's workloads
    "register_cfg1": (128, 1, 2048, 2048, 0, 2048, 0x5EED, 16),
    "register_cfg4": (256, 3, 4000, 6000, 1, 2048, 0x5EED, 16),
}


def correlate(ref_f, img):
    """real correlation plane (numpy scaling 1/S^2 -- a positive factor, same arg-max)"""
    S = img.shape[0]
    return np.fft.irfft2(ref_f * np.conj(np.fft.rfft2(img.astype(np.float64))), s=(S, S))


def make(name, N, C, H, W, layer, S, seed, maxshift):
    y0, x0 = (H - S) // 2, (W - S) // 2
    t0 = time.time()
    sel = orc.synth_window(N, layer, y0, x0, S, S, seed=seed, maxshift=maxshift)
    ref_f = np.fft.rfft2(sel[0].astype(np.float64))
    sx = np.zeros(N, np.int32)
    sy = np.zeros(N, np.int32)
    margin = np.full(N, np.inf)
    for f in range(1, N):
        c = correlate(ref_f, sel[f])
        k = int(np.argmax(c))
        c.flat[k] = -np.inf
        k2 = int(np.argmax(c))
        ky, kx = divmod(k, S)
        ky2, kx2 = divmod(k2, S)
        e1 = orc.xcorr_at(sel[0], sel[f], ky, kx)
        e2 = orc.xcorr_at(sel[0], sel[f], ky2, kx2)
        assert e1 > e2, (f, e1, e2)
        margin[f] = (e1 - e2) / e1
        sy[f] = ky - S if ky > S // 2 else ky
        sx[f] = kx - S if kx > S // 2 else kx
    q = np.array([orc.quality(sel[f]) for f in range(N)])
    ex, ey = orc.synth_shifts(N, seed=seed, maxshift=maxshift)
    assert np.array_equal(sx, ex) and np.array_equal(sy, ey), "registration does not recover the translations"
    out = os.path.join(HERE, name + ".npz")
    np.savez_compressed(out, shiftx=sx, shifty=sy, quality_raw=q, margin=margin,
                        geometry=np.array([N, C, H, W, layer, S, y0, x0, seed, maxshift], np.int64))
    print(f"{name}: {N} frames S={S} in {time.time() - t0:.0f} s, min relative margin {margin[1:].min():.3e}")


if __name__ == "__main__":
    for name, cfg in CONFIGS.items():
        make(name, *cfg)
