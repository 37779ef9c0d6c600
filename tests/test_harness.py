"""The reference-side binding compiled and exercised: harness/siril_glue.c holds the bodies of
stack_summing / stack_mean_with_rejection / stack_median / stack_addmax / stack_addmin and
register_shift_dft with the reference's signatures (struct stacking_args *,
struct registration_args *, restated GTK-free in harness/siril_compat.h), calling
libsirilgpu.so.  harness_stack() builds struct stacking_args the way start_stacking
(src/stacking/stacking.c:1871-1927) does and calls args->method(&args) from C; the result is
read back from gfit (the ownership hand-off of :1820-1827) and compared with the oracle."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import harness_lib as hl
import oracle_lib as orc
from seq_files import write_fits, write_ser

SUM, MEAN, MEDIAN, MAX, MIN = 0, 1, 2, 3, 4
NO_REJEC, PERCENTILE, SIGMA, SIGMEDIAN, WINSORIZED, LINEARFIT = range(6)


def test_harness_builds_and_exports():
    """CPU: the glue and its environment link against libsirilgpu.so and export the
    reference's entry points"""
    lib = hl.load()
    for name in ["stack_summing", "stack_mean_with_rejection", "stack_median", "stack_addmax", "stack_addmin",
                 "register_shift_dft", "seq_opened_read_region", "seq_read_frame_part", "compute_normalization"]:
        assert hasattr(lib, name), name
    assert os.path.exists(hl.CLI)


def _seq_files(tmp_path, frames, fmt):
    if fmt == "ser":
        p = str(tmp_path / "h.ser")
        write_ser(p, frames, depth=16)
        return hl.Sequence.ser(p)
    paths = []
    for i in range(frames.shape[0]):
        p = str(tmp_path / f"h_{i + 1:05d}.fit")
        write_fits(p, frames[i])
        paths.append(p)
    return hl.Sequence.fits(paths)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["ser", "fits"])
@pytest.mark.parametrize("rejection", [SIGMA, WINSORIZED, LINEARFIT, NO_REJEC])
def test_stack_mean_with_rejection_from_c(tmp_path, fmt, rejection):
    """stack_mean_with_rejection(&args) called from C with registration shifts on the
    registration layer and 3 of 20 frames excluded (stack_filter_included) == the oracle on
    the included frames"""
    lib = hl.load()
    N, C, H, W = 20, 1, 40, 72
    frames = orc.synth(N, C, H, W, seed=90 + rejection, maxshift=5)
    sx, sy = orc.synth_shifts(N, seed=90 + rejection, maxshift=5)
    excl = [3, 11, 17]
    keep = [i for i in range(N) if i not in excl]
    sig = (3.0, 3.0)
    rc, ref, _ = orc.stack_rejection(frames[keep], rejection, sig=sig, shiftx=sx[keep], shifty=sy[keep],
                                     max_thread=4)
    assert rc == 0
    lib.harness_set_max_thread(4)
    with _seq_files(tmp_path, frames, fmt) as seq:
        for i in excl:
            lib.harness_set_included(seq.h, i, 0)
        seq.set_regdata(0, sx, sy)
        lib.harness_set_registration_layer(0)
        rc = lib.harness_stack(seq.h, MEAN, rejection, 0, sig[0], sig[1], 1, 0)
        lib.harness_set_registration_layer(-1)
        assert rc == 0
        assert np.array_equal(hl.gfit(), ref)


@pytest.mark.gpu
def test_stack_summing_median_max_min_from_c(tmp_path):
    """stack_summing (gfit.hi = the sum maximum), stack_median with additive + scaling
    normalisation from statistics computed on the GPU, stack_addmax / stack_addmin"""
    lib = hl.load()
    N, C, H, W = 12, 1, 32, 48
    frames = orc.synth(N, C, H, W, seed=7, maxshift=4)
    sx, sy = orc.synth_shifts(N, seed=7, maxshift=4)
    with _seq_files(tmp_path, frames, "fits") as seq:
        seq.set_regdata(0, sx, sy)
        lib.harness_set_registration_layer(0)
        assert lib.harness_stack(seq.h, SUM, 0, 0, 0.0, 0.0, 0, 0) == 0
        rc, ref, mref = orc.stack_sum(frames, sx, sy)
        assert np.array_equal(hl.gfit(), ref) and lib.harness_gfit_hi() == min(mref, 65535)
        for m, is_max in [(MAX, True), (MIN, False)]:
            assert lib.harness_stack(seq.h, m, 0, 0, 0.0, 0.0, 0, 0) == 0
            rc, ref = orc.stack_maxmin(frames, is_max, sx, sy)
            assert np.array_equal(hl.gfit(), ref)
        lib.harness_set_registration_layer(-1)
        # median with ADDITIVE_SCALING: statistics of each frame (IKSS, layer 0) as the oracle
        loc = np.zeros(N)
        scl = np.zeros(N)
        for i in range(N):
            rcs, loc[i], scl[i] = orc.statistics_ikss(frames[i])
            assert rcs == 0
        off, mul, sc = orc.compute_normalization(3, loc, scl)
        rc, ref = orc.stack_median(frames, normalize=3, offset=off, mul=mul, scale=sc, max_thread=4)
        assert lib.harness_stack(seq.h, MEDIAN, 0, 3, 0.0, 0.0, 0, 0) == 0
        assert np.array_equal(hl.gfit(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["ser", "fits"])
def test_register_shift_dft_from_c(tmp_path, fmt):
    """register_shift_dft(&args) from C: selections read with seq_read_frame_part (FITS one row
    lower than SER, readfits_partial :512), shifts and normalised qualities == the oracle on the
    selections the reference would read; frames excluded keep zero regdata"""
    lib = hl.load()
    N, C, H, W, S = 9, 1, 80, 96, 64
    frames = orc.synth(N, C, H, W, seed=23, maxshift=5)
    frames[:, :, 30:35, 40:45] = 40000  # structure for QualityEstimate (a 3x3 spot gives NaN
                                        # qualities on the FITS selection, GPU and oracle alike)
    x, y = 10, 6                        # display coordinates of the selection
    m0 = H - y - S - (1 if fmt == "fits" else 0)     # its first memory row
    sel = frames[:, 0, m0:m0 + S, x:x + S]
    inc = np.ones(N, np.int32)
    inc[4] = 0
    rx, ry, rq = orc.register_dft(sel, ref_image=2, included=inc)
    with _seq_files(tmp_path, frames, fmt) as seq:
        lib.harness_set_reference_image(seq.h, 2)
        lib.harness_set_included(seq.h, 4, 0)
        assert lib.harness_register(seq.h, 0, x, y, S, 0) == 0
        gx, gy, gq = seq.regdata(0, N)
    m = inc.astype(bool)
    assert np.array_equal(gx[m], rx[m]) and np.array_equal(gy[m], ry[m])
    assert np.array_equal(gq[m], rq[m], equal_nan=True)
    assert not np.isnan(rq[m]).all()                # the bright spot gives a real quality map
    assert gx[4] == 0 and gy[4] == 0 and gq[4] == 0


@pytest.mark.gpu
def test_register_fits_selection_touching_bottom_fails(tmp_path):
    """a selection touching the bottom display row: fpixel[1] = 0 on FITS -> the read and the
    registration fail (the reference's behaviour), while SER registers"""
    lib = hl.load()
    N, H, W, S = 4, 64, 64, 32
    frames = orc.synth(N, 1, H, W, seed=5, maxshift=3)
    with _seq_files(tmp_path, frames, "fits") as seq:
        assert lib.harness_register(seq.h, 0, 0, H - S, S, 1) != 0
    with _seq_files(tmp_path, frames, "ser") as seq:
        assert lib.harness_register(seq.h, 0, 0, H - S, S, 1) == 0


def _star_field(N, H, W, seed, maxshift):
    """frames of one star field translated by up to maxshift pixels, plus noise: registrable by
    the DFT on a 64-pixel selection (the plain synthetic noise is not, and its arg-max shifts
    exceed the oracle's block-height guard)"""
    rng = np.random.default_rng(seed)
    m = maxshift + 2
    yy, xx = np.mgrid[0:H + 2 * m, 0:W + 2 * m]
    base = np.full(yy.shape, 1200.0)
    for _ in range(40):
        cy, cx = rng.uniform(0, H + 2 * m), rng.uniform(0, W + 2 * m)
        a, s = rng.uniform(2000, 20000), rng.uniform(1.0, 2.5)
        base += a * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * s * s))
    dx, dy = rng.integers(-maxshift, maxshift + 1, N), rng.integers(-maxshift, maxshift + 1, N)
    dx[0] = dy[0] = 0
    frames = np.zeros((N, 1, H, W), np.uint16)
    for f in range(N):
        im = base[m + dy[f]:m + dy[f] + H, m + dx[f]:m + dx[f] + W] + rng.normal(0, 30, (H, W))
        frames[f, 0] = np.clip(np.rint(im), 0, 65535)
    return frames


@pytest.mark.gpu
def test_cli_register_and_stack(tmp_path):
    """siril_cli: open a SER, register layer 0 on a centred selection, sigma-clip stack with
    the shifts, save the FITS: the saved image == the oracle with the oracle's shifts"""
    N, H, W, S = 16, 96, 128, 64
    frames = _star_field(N, H, W, seed=61, maxshift=4)
    p = str(tmp_path / "c.ser")
    write_ser(p, frames, depth=16)
    x, y = (W - S) // 2, (H - S) // 2
    m0 = H - y - S
    rx, ry, _ = orc.register_dft(frames[:, 0, m0:m0 + S, x:x + S])
    assert np.abs(rx).max() <= 5 and np.abs(ry).max() <= 5     # a real registration
    rc, ref, _ = orc.stack_rejection(frames, SIGMA, sig=(4.0, 3.0), shiftx=rx, shifty=ry, max_thread=16)
    out = str(tmp_path / "out.fit")
    r = subprocess.run([hl.CLI, "--ser", p, "--register", "0", str(x), str(y), str(S), "--stack", "mean",
                        "--rejection", "sigma", "--sig", "4", "3", "-o", out], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    import sirilgpu as sg
    with sg.Seq.open_fits([out]) as s:
        got = s.read_frame(0)
    bad = np.argwhere(got != ref)
    assert len(bad) == 0, (len(bad), bad[:8].tolist(), r.stdout, rx.tolist(), ry.tolist())


def _rej_logged(text, C):
    """the per-channel rejection percentages the glue logs (:1811-1817 format)"""
    import re
    got = re.findall(r"Pixel rejection in channel #(\d+): ([0-9.]+)% - ([0-9.]+)%", text)
    return [(float(a), float(b)) for _, a, b in got[-C:]]


@pytest.mark.gpu
@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_multi_device_slots_from_c(tmp_path, capfd, devs):
    """the glue's context on several device slots (sg_init(ndev, {0, 0, ...}) on one card): every
    slot stacks its share of the rows from its own host thread with its own readers.  SIGMA and
    WINSORIZED rejection (result + logged rejection %), SUM with the 65535/max scaling over the
    whole image (gfit.hi), MEDIAN with normalisation == the oracle; gfit.exposure = the EXPTIME
    sum (EXPOSURE where EXPTIME is missing or <= 0, :1284-1294) for the rejection / median
    stackers and readfits' carried value for the sum stackers"""
    lib = hl.load()
    N, C, H, W = 14, 3, 37, 70
    frames = orc.synth(N, C, H, W, seed=33, maxshift=4)
    sx, sy = orc.synth_shifts(N, seed=33, maxshift=4)
    exptime = [("EXPTIME", f"{1.5 * (i + 1)}") if i % 4 else ("EXPOSURE", f"{2.0 + i}") for i in range(N)]
    exptime[5] = ("EXPTIME", "0.")          # <= 0: the rejection stackers fall back to EXPOSURE
    paths = []
    for i in range(N):
        p = str(tmp_path / f"m_{i + 1:05d}.fit")
        keys = [exptime[i]] + ([("EXPOSURE", "7.25")] if i == 5 else [])
        write_fits(p, frames[i], keys=keys)
        paths.append(p)
    exp_rej = sum(float(v) if not (k == "EXPTIME" and float(v) <= 0) else 7.25 for k, v in exptime)
    exp_sum = sum(float(v) for k, v in exptime)      # readfits takes EXPTIME even at 0
    try:
        assert hl.set_devices(devs) == 0
        lib.harness_set_max_thread(4)
        with hl.Sequence.fits(paths) as seq:
            seq.set_regdata(0, sx, sy)
            lib.harness_set_registration_layer(0)
            for rejection, sig in [(SIGMA, (3.0, 3.0)), (WINSORIZED, (2.5, 2.5))]:
                capfd.readouterr()
                assert lib.harness_stack(seq.h, MEAN, rejection, 0, sig[0], sig[1], 0, 0) == 0
                out = capfd.readouterr().out
                rc, ref, rej = orc.stack_rejection(frames, rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=4)
                assert np.array_equal(hl.gfit(), ref), rejection
                nb_tot = float(W * H * N)
                want = [(round(rej[c][0] / nb_tot * 100.0, 3), round(rej[c][1] / nb_tot * 100.0, 3)) for c in range(C)]
                assert _rej_logged(out, C) == want, (out, want)
                assert lib.harness_gfit_exposure() == pytest.approx(exp_rej, rel=0, abs=1e-9)
            assert lib.harness_stack(seq.h, SUM, 0, 0, 0.0, 0.0, 0, 0) == 0
            rc, ref, mref = orc.stack_sum(frames, sx, sy)
            assert mref > 65535
            assert np.array_equal(hl.gfit(), ref) and lib.harness_gfit_hi() == 65535
            assert lib.harness_gfit_exposure() == pytest.approx(exp_sum, rel=0, abs=1e-9)
            lib.harness_set_registration_layer(-1)
            loc, scl = np.zeros(N), np.zeros(N)
            for i in range(N):
                _, loc[i], scl[i] = orc.statistics_ikss(frames[i])
            off, mul, sc = orc.compute_normalization(2, loc, scl)
            rc, ref = orc.stack_median(frames, normalize=2, offset=off, mul=mul, scale=sc, max_thread=4)
            assert lib.harness_stack(seq.h, MEDIAN, 0, 2, 0.0, 0.0, 0, 0) == 0
            assert np.array_equal(hl.gfit(), ref)
    finally:
        lib.harness_set_registration_layer(-1)
        hl.set_devices(None)


@pytest.mark.gpu
@pytest.mark.parametrize("devs", [None, [0, 0]])
def test_register_cancel_from_c(tmp_path, devs):
    """register_shift_dft with run_in_thread and get_thread_run() turning false after 3 polls:
    the reference polls every frame index before its reference / inclusion checks (:280-290),
    registers the frames polled before the failing poll, still returns 0, keeps
    the rest's regdata and skips normalizeQualityData (:166-168), so the registered frames keep
    RAW qualities; the best frame is logged"""
    lib = hl.load()
    N, H, W, S = 9, 96, 128, 64
    frames = _star_field(N, H, W, seed=17, maxshift=4)
    x, y = (W - S) // 2, (H - S) // 2
    m0 = H - y - S
    sel = frames[:, 0, m0:m0 + S, x:x + S]
    ref = 2
    done = [0, 1]                          # polls 1, 2 (frames 0, 1), 3 (frame 2 = ref, skipped); frame 3's fails
    inc = np.zeros(N, np.int32)
    inc[done] = 1
    rx, ry, _ = orc.register_dft(sel, ref_image=ref, included=inc)
    p = str(tmp_path / "c.ser")
    write_ser(p, frames, depth=16)
    try:
        if devs:
            assert hl.set_devices(devs) == 0
        with hl.Sequence.ser(p) as seq:
            lib.harness_set_reference_image(seq.h, ref)
            seq.set_regdata(0, np.full(N, 7), np.full(N, -7))     # earlier registration data
            lib.harness_set_run_in_thread(1)
            lib.harness_set_cancel_after(3)
            rc = lib.harness_register(seq.h, 0, x, y, S, 1)
            lib.harness_set_cancel_after(-1)
            lib.harness_set_run_in_thread(0)
            assert rc == 0
            gx, gy, gq = seq.regdata(0, N)
        for f in range(N):
            if f in done or f == ref:
                assert (gx[f], gy[f]) == ((rx[f], ry[f]) if f != ref else (0, 0)), f
                assert gq[f] == orc.quality(sel[f]), f      # raw QualityEstimate
            else:
                assert (gx[f], gy[f]) == (7, -7), f         # kept
    finally:
        lib.harness_set_cancel_after(-1)
        lib.harness_set_run_in_thread(0)
        if devs:
            hl.set_devices(None)


@pytest.mark.gpu
@pytest.mark.parametrize("existing", [False, True])
@pytest.mark.parametrize("bad", [7, 70, 0])
def test_register_read_failure(tmp_path, capfd, existing, bad):
    """one unreadable frame (seq_read_frame_part fails): register_shift_dft returns the failure,
    the layer's registration array is freed and seq->regparam[layer] is NULL afterwards, whether
    it was new or the existing one being recomputed (:375-381; the reference frame's failure
    :238-244 frees it too), no 'Registration finished' is logged; an existing array's reuse is
    logged as 'Recomputing already existing registration' (:213-216).  bad = 70 fails in the
    second batch handed to the library, bad = 0 is the reference frame"""
    lib = hl.load()
    N, H, W, S = 80, 64, 64, 32
    frames = orc.synth(N, 1, H, W, seed=19, maxshift=3)
    p = str(tmp_path / "f.ser")
    write_ser(p, frames, depth=16)
    with hl.Sequence.ser(p) as seq:
        if existing:
            seq.set_regdata(0, np.arange(N, dtype=np.int32) % 5, -(np.arange(N, dtype=np.int32) % 3))
        lib.harness_set_fail_read(bad)
        try:
            capfd.readouterr()
            rc = lib.harness_register(seq.h, 0, 16, 16, S, 1)
            out = capfd.readouterr().out
        finally:
            lib.harness_set_fail_read(-1)
        assert rc == 1
        assert seq.regdata(0, N) is None            # seq->regparam[0] == NULL
        assert ("Recomputing already existing registration for this layer" in out) == existing, out
        assert "Registration finished" not in out
        if bad == 0:
            assert "could not load first image to register, aborting" in out, out
        else:
            assert f"Could not load partial image {bad}" in out, out
        # the sequence registers again once the frame reads (a new array, no 'Recomputing')
        capfd.readouterr()
        assert lib.harness_register(seq.h, 0, 16, 16, S, 1) == 0
        out = capfd.readouterr().out
        assert "Recomputing" not in out and "Registration finished" in out
        sel = frames[:, 0, H - 16 - S:H - 16, 16:16 + S]
        rx, ry, _ = orc.register_dft(sel)
        gx, gy, _ = seq.regdata(0, N)
        assert np.array_equal(gx, rx) and np.array_equal(gy, ry)


@pytest.mark.gpu
def test_register_best_frame_logged(tmp_path, capfd):
    """the best frame (q_index, :315-324, logged :397) is the frame of highest quality"""
    lib = hl.load()
    N, H, W, S = 6, 96, 128, 64
    frames = _star_field(N, H, W, seed=29, maxshift=3)
    x, y = (W - S) // 2, (H - S) // 2
    m0 = H - y - S
    sel = frames[:, 0, m0:m0 + S, x:x + S]
    q = [orc.quality(sel[f]) for f in range(N)]
    want = 0
    for f in range(1, N):
        if q[f] > q[want]:
            want = f
    p = str(tmp_path / "b.ser")
    write_ser(p, frames, depth=16)
    with hl.Sequence.ser(p) as seq:
        capfd.readouterr()
        assert lib.harness_register(seq.h, 0, x, y, S, 1) == 0
        out = capfd.readouterr().out
    assert f"Best frame: #{want}." in out, out
