"""Generate the committed golden fixtures (tests/golden/*.npz).

The reference publishes no test vectors and cannot be built here, so
these vectors are produced by the C oracle (oracle/, restatement of the reference
stackers) and each one is cross-checked at generation time against the independent
numpy restatement (tests/oracle_numpy.py).  Cases follow SURVEY.md §8c "Fixtures that
must exist".  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as orc          # noqa: E402
import oracle_numpy as onp        # noqa: E402

SIG = {1: (0.2, 0.1), 2: (4.0, 3.0), 3: (4.0, 3.0), 4: (4.0, 3.0), 5: (5.0, 5.0)}


def noisy(rng, N, C, H, W, lo=900, hi=1100, p_hot=0.06, p_cold=0.04):
    f = rng.integers(lo, hi, size=(N, C, H, W)).astype(np.uint16)
    m = rng.random(f.shape)
    f[m < p_hot] = 65535
    f[m > 1 - p_cold] = 0
    return f


def main():
    rng = np.random.default_rng(20261015)
    cases = {}
    # rejection modes on synthetic scene with shifts (out-of-frame zeros participate)
    for rej in (0, 1, 2, 3, 4, 5):
        N, C, H, W = 16, 1, 24, 40
        fr = orc.synth(N, C, H, W, seed=100 + rej, maxshift=5)
        sx, sy = orc.synth_shifts(N, seed=100 + rej, maxshift=5)
        sig = SIG.get(rej, (4.0, 3.0))
        rc, out, rj = orc.stack_rejection(fr, rej, sig=sig, shiftx=sx, shifty=sy, max_thread=1)
        nout, nrj = onp.stack_rejection_1thread(fr, rej, sig, sx, sy)
        assert rc == 0 and np.array_equal(out, nout) and np.array_equal(rj, nrj), rej
        cases[f"rej{rej}_synth"] = dict(kind="rejection", frames=fr, shiftx=sx, shifty=sy,
                                        rejection=rej, sig=np.array(sig), max_thread=1, out=out, rej=rj)
    # small N: early break + stale rejected[] carried across pixels (SURVEY a3 iii)
    for N in (3, 4, 5, 6, 8):
        for rej in (2, 4, 5):
            fr = noisy(rng, N, 1, 6, 24)
            rc, out, rj = orc.stack_rejection(fr, rej, sig=(1.0, 1.0), max_thread=1)
            nout, nrj = onp.stack_rejection_1thread(fr, rej, (1.0, 1.0))
            assert rc == 0 and np.array_equal(out, nout) and np.array_equal(rj, nrj), (N, rej)
            cases[f"rej{rej}_smallN{N}"] = dict(kind="rejection", frames=fr, rejection=rej,
                                                sig=np.array((1.0, 1.0)), max_thread=1, out=out, rej=rj)
    # constant stacks: sigma == 0 (Winsorized 0/0 exit), knife-edge integer patterns
    fr = np.full((16, 1, 4, 16), 1234, dtype=np.uint16)
    fr[:, 0, 1, :] = np.array([1000] * 8 + [1010] * 8, dtype=np.uint16)[:, None]
    fr[:, 0, 2, :] = np.array(list(range(1000, 1016)), dtype=np.uint16)[:, None]
    fr[:, 0, 3, :] = np.array([0] * 15 + [65535], dtype=np.uint16)[:, None]
    for rej in (2, 3, 4, 5):
        rc, out, rj = orc.stack_rejection(fr, rej, sig=(2.0, 1.5), max_thread=1)
        nout, nrj = onp.stack_rejection_1thread(fr, rej, (2.0, 1.5))
        assert rc == 0 and np.array_equal(out, nout) and np.array_equal(rj, nrj), rej
        cases[f"rej{rej}_edges"] = dict(kind="rejection", frames=fr, rejection=rej,
                                        sig=np.array((2.0, 1.5)), max_thread=1, out=out, rej=rj)
    # median: even N truncation of (a+b)/2
    for N in (7, 10):
        fr = noisy(rng, N, 3, 8, 20)
        rc, out = orc.stack_median(fr)
        assert rc == 0 and np.array_equal(out, onp.stack_median(fr))
        cases[f"median_N{N}"] = dict(kind="median", frames=fr, out=out)
    # sum: pixel 0 never accumulated, 65535/max scaling; and the ratio == 1 branch
    fr = orc.synth(16, 1, 24, 32, seed=5, maxshift=6)
    sx, sy = orc.synth_shifts(16, seed=5, maxshift=6)
    rc, out, mx = orc.stack_sum(fr, sx, sy)
    nout, nmx = onp.stack_summing(fr, sx, sy)
    assert np.array_equal(out, nout) and mx == nmx
    cases["sum_scaled"] = dict(kind="sum", frames=fr, shiftx=sx, shifty=sy, out=out, maxim=np.array(mx))
    fr = np.full((3, 1, 5, 7), 100, dtype=np.uint16)
    rc, out, mx = orc.stack_sum(fr)
    nout, nmx = onp.stack_summing(fr)
    assert np.array_equal(out, nout) and mx == nmx == 300
    cases["sum_unscaled"] = dict(kind="sum", frames=fr, out=out, maxim=np.array(mx))
    # max / min
    for is_max in (True, False):
        rc, out = orc.stack_maxmin(cases["sum_scaled"]["frames"], is_max, sx, sy)
        cases["max" if is_max else "min"] = dict(kind="max" if is_max else "min",
                                                 frames=cases["sum_scaled"]["frames"],
                                                 shiftx=sx, shifty=sy, out=out)
    # quality estimate (registration): star field and an all-dark frame (NaN)
    img = orc.synth(1, 1, 64, 64, seed=77, maxshift=0)[0, 0].copy()
    img[30:34, 30:34] = 30000
    q = orc.quality(img)
    assert q == onp.quality(img), (q, onp.quality(img))
    cases["quality_star"] = dict(kind="quality", img=img, q=np.array(q))
    dark = np.zeros((40, 40), dtype=np.uint16)   # max == 0: no stretch, no pixel >= 10240
    qd = orc.quality(dark)
    assert np.isnan(qd) and np.isnan(onp.quality(dark))
    cases["quality_dark"] = dict(kind="quality", img=dark, q=np.array(qd))
    # DFT registration on small power-of-two selections
    sel = orc.synth(6, 1, 64, 64, seed=31, maxshift=7)[:, 0].copy()
    sx, sy, qq = orc.register_dft(sel)
    cases["register_dft64"] = dict(kind="register", sel=sel, shiftx=sx, shifty=sy, quality=qq)
    for name, d in cases.items():
        d = {k: (np.asarray(v) if not isinstance(v, str) else np.array(v)) for k, v in d.items()}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(f"wrote {len(cases)} fixtures")


if __name__ == "__main__":
    main()
