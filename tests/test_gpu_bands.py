"""Row bands through the C ABI (sg_stack_u16_device with row_begin > 0, and the host-pull
path streaming a sequence larger than its HBM budget in row bands).

Row bands are the multi-GPU shard of the stackers (the reference's own block
scheme, src/stacking/stacking.c:1397-1476).  Every band result must equal the full-image
oracle restricted to the band, bit for bit, including the stale rejected[] a band's first
pixel inherits from the previous pixel of the reference's OpenMP thread (§8a a3 iii) when
its first sigma pass breaks early (`N - r <= 4`, :1684).  With only the band and the rows
its shifts reach resident, such a pixel's predecessor cannot be recomputed: the call must
fail loudly rather than guess.
"""
import os

import numpy as np
import pytest

import oracle_lib as orc
import sirilgpu as sg
import sirilgpu_dist as sd
from test_gpu_stack import REJ, assert_same

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda()
    torch.cuda.synchronize()        # the library runs on its own (non-blocking) stream
    return t


def _oracle(frames, method, rejection, sig, sx, sy, max_thread):
    if method == sg.MEAN:
        rc, ref, rej = orc.stack_rejection(frames, rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=max_thread)
    elif method == sg.MEDIAN:
        rc, ref = orc.stack_median(frames, max_thread=max_thread)
        rej = np.zeros((3, 2), np.uint64)
    else:
        rc, ref = orc.stack_maxmin(frames, method == sg.MAX, sx, sy)
        rej = np.zeros((3, 2), np.uint64)
    assert rc == 0
    return ref, rej


def _halo(b, e, H, sy):
    lo = max(0, b - int(sy.max()))
    hi = min(H - 1, e - 1 - int(sy.min()))
    return lo, hi


def _stack_bands(ctx, frames, method, rejection, sig, sx, sy, max_thread, world, resident="full"):
    """stack every band [b, e) of `world` bands with one device call each; resident = "full"
    (all frame rows in HBM) or "band" (only the rows the band reads, biased base pointer)"""
    import torch
    N, C, H, W = frames.shape
    d_out = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()        # the zero fill must land before the library's stream writes
    rej = np.zeros((3, 2), np.uint64)
    full = _dev(frames) if resident == "full" else None
    for r in range(world):
        b, e = sd.row_band(r, world, H)
        if resident == "full":
            desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                                      max_thread=max_thread, max_number_of_rows=H)
            rj, _ = ctx.stack_device(desc, full.data_ptr(), C * H * W, H * W, d_out.data_ptr(), b, e)
        else:
            lo, hi = _halo(b, e, H, sy if method != sg.MEDIAN else np.zeros(1, np.int32))
            nres = hi - lo + 1
            band = _dev(frames[:, :, lo:hi + 1])
            desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                                      max_thread=max_thread, max_number_of_rows=H, resident_rows=(lo, hi + 1))
            base = band.data_ptr() - lo * W * 2
            rj, _ = ctx.stack_device(desc, base, C * nres * W, nres * W, d_out.data_ptr(), b, e)
        rej += rj
    torch.cuda.synchronize()
    return d_out.cpu().numpy().view(np.uint16).reshape(C, H, W), rej


CASES = [(sg.MEAN, sg.SIGMA), (sg.MEAN, sg.WINSORIZED), (sg.MEAN, sg.PERCENTILE), (sg.MEAN, sg.SIGMEDIAN),
         (sg.MEAN, sg.LINEARFIT), (sg.MEAN, sg.NO_REJEC), (sg.MEDIAN, sg.NO_REJEC), (sg.MAX, sg.NO_REJEC),
         (sg.MIN, sg.NO_REJEC)]


@pytest.mark.parametrize("resident", ["full", "band"])
@pytest.mark.parametrize("method,rejection", CASES)
def test_bands_match_full_image(gpu_ctx, method, rejection, resident):
    """synthetic scene with registration shifts, 3 bands (the histogram path at N = 24)"""
    N, C, H, W = 24, 2, 40, 150
    frames = orc.synth(N, C, H, W, seed=31, maxshift=6)
    sx, sy = orc.synth_shifts(N, seed=31, maxshift=6)
    sig = REJ[rejection]
    ref, rej_ref = _oracle(frames, method, rejection, sig, sx, sy, 4)
    out, rej = _stack_bands(gpu_ctx, frames, method, rejection, sig, sx, sy, 4, 3, resident)
    assert_same(out, ref, f"bands method={method} rej={rejection} resident={resident}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


def _early_break_frames(world, H, W, N=6, seed=5):
    """the first pixel of every band but the last (thread order: top row, x = 0) breaks early
    in its first pass and inherits its predecessor's rejected[5] = 1 (tests/test_dist_gloo.py)"""
    rng = np.random.default_rng(seed)
    frames = rng.integers(900, 1100, size=(N, 1, H, W)).astype(np.uint16)
    m = rng.random(frames.shape)
    frames[m < 0.1] = 65535
    frames[m > 0.9] = 0
    for r in range(world - 1):
        b, e = sd.row_band(r, world, H)
        frames[:, 0, e - 1, 0] = [0, 0, 1000, 1010, 1020, 1100]
        frames[:, 0, e, W - 1] = [1000, 1000, 1000, 1000, 1000, 65535]
    return frames


@pytest.mark.parametrize("max_thread", [1, 2])
@pytest.mark.parametrize("world", [2, 3])
def test_band_first_pixel_inherits_stale_state(gpu_ctx, world, max_thread):
    H, W, N = 12, 70, 6
    frames = _early_break_frames(world, H, W, N)
    sx = sy = np.zeros(N, np.int32)
    sig = (1.0, 1.0)
    ref, rej_ref = _oracle(frames, sg.MEAN, sg.SIGMA, sig, sx, sy, max_thread)
    out, rej = _stack_bands(gpu_ctx, frames, sg.MEAN, sg.SIGMA, sig, sx, sy, max_thread, world, "full")
    assert_same(out, ref, f"early-break bands world={world} thr={max_thread}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    # the planted pixel really depends on its out-of-band predecessor
    b, e = sd.row_band(0, world, H)
    assert ref[0, e - 1, 0] == round((1000 + 1010 + 1020) / 3) or max_thread > 1


def test_band_stale_state_needs_resident_rows(gpu_ctx):
    """band-only residency: the inherited state of the band's first pixel would need rows
    outside the band -> SG_ERR_GENERIC with a message, never a guess or an out-of-bounds read"""
    import torch
    world, H, W, N = 2, 12, 70, 6
    frames = _early_break_frames(world, H, W, N)
    z = np.zeros(N, np.int32)
    b, e = sd.row_band(0, world, H)
    band = _dev(frames[:, :, b:e])
    d_out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=(1.0, 1.0), shiftx=z, shifty=z,
                              max_thread=1, max_number_of_rows=H, resident_rows=(b, e))
    with pytest.raises(RuntimeError, match="resident"):
        gpu_ctx.stack_device(desc, band.data_ptr() - b * W * 2, (e - b) * W, (e - b) * W, d_out.data_ptr(), b, e)


def test_band_rows_not_resident_rejected(gpu_ctx):
    """a resident range that misses rows the band's shifts reach is refused up front"""
    import torch
    N, C, H, W = 16, 1, 32, 64
    frames = orc.synth(N, C, H, W, seed=3, maxshift=4)
    sx, sy = orc.synth_shifts(N, seed=3, maxshift=4)
    b, e = 10, 20
    band = _dev(frames[:, :, b:e])          # no halo
    d_out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.SIGMA, shiftx=sx, shifty=sy,
                              max_number_of_rows=H, resident_rows=(b, e))
    with pytest.raises(RuntimeError, match="not all resident"):
        gpu_ctx.stack_device(desc, band.data_ptr() - b * W * 2, (e - b) * W, (e - b) * W, d_out.data_ptr(), b, e)


def _with_budget(nbytes, fn, devices=None):
    """fn(ctx) on a context created under the budget knob (knobs are read at sg_init)"""
    old = os.environ.get("SG_HOST_BUDGET_BYTES")
    os.environ["SG_HOST_BUDGET_BYTES"] = str(nbytes)
    try:
        with sg.Context(devices) as ctx:
            return fn(ctx)
    finally:
        if old is None:
            del os.environ["SG_HOST_BUDGET_BYTES"]
        else:
            os.environ["SG_HOST_BUDGET_BYTES"] = old


@pytest.mark.parametrize("method,rejection", CASES + [(sg.SUM, sg.NO_REJEC)])
@pytest.mark.parametrize("band_rows", [1, 7])
def test_host_pull_streams_row_bands(gpu_ctx, method, rejection, band_rows):
    """a budget of `band_rows` rows (+ the shift halo) per frame: the host-pull path reads the
    sequence through the region callback band by band, as the reference's row blocks do"""
    N, C, H, W = 20, 2, 30, 90
    frames = orc.synth(N, C, H, W, seed=41, maxshift=5)
    sx, sy = orc.synth_shifts(N, seed=41, maxshift=5)
    sig = REJ[rejection]
    if method == sg.SUM:
        rc, ref, mref = orc.stack_sum(frames, sx, sy)
        assert rc == 0 and mref > 65535     # the 65535/max scaling over the whole image
        rej_ref = np.zeros((3, 2), np.uint64)
    else:
        ref, rej_ref = _oracle(frames, method, rejection, sig, sx, sy, 4)
    halo = 0 if method == sg.MEDIAN else int(sy.max() - sy.min())
    budget = N * C * W * 2 * (band_rows + halo)
    desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=4, max_number_of_rows=H)
    rc, out, rej, maxim, err = _with_budget(budget, lambda c: c.stack_host(desc, frames) + (c.error(),))
    assert rc == 0, err
    assert_same(out, ref, f"host bands method={method} rej={rejection} rows={band_rows}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if method == sg.SUM:
        assert maxim == mref


def _with_env(env, fn):
    """fn(ctx) on a context created under the given knobs (read at sg_init)"""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        with sg.Context() as ctx:
            return fn(ctx)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.mark.parametrize("method,rejection", CASES)
@pytest.mark.parametrize("overlap", [1, 0])
def test_host_pull_overlapped_bands(gpu_ctx, method, rejection, overlap):
    """a budget of two bands of 4 rows (+ halo): band k + 1 is read into the second frame buffer
    while band k stacks (SG_PULL_OVERLAP=1, the default) over >= 3 bands; the image and the
    counters equal the oracle's, as with the bands read and stacked one after the other"""
    N, C, H, W = 24, 2, 40, 96
    frames = orc.synth(N, C, H, W, seed=43, maxshift=4)
    sx, sy = orc.synth_shifts(N, seed=43, maxshift=4)
    sig = REJ[rejection]
    ref, rej_ref = _oracle(frames, method, rejection, sig, sx, sy, 4)
    halo = 0 if method == sg.MEDIAN else int(sy.max() - sy.min())
    budget = N * C * W * 2 * 2 * (4 + halo)
    desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=4, max_number_of_rows=H)
    rc, out, rej, _, err = _with_env({"SG_HOST_BUDGET_BYTES": budget, "SG_PULL_OVERLAP": overlap},
                                     lambda c: c.stack_host(desc, frames) + (c.error(),))
    assert rc == 0, err
    assert_same(out, ref, f"overlapped host bands method={method} rej={rejection} overlap={overlap}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


def test_host_pull_budget_too_small(gpu_ctx):
    N, C, H, W = 8, 1, 16, 32
    frames = orc.synth(N, C, H, W, seed=2, maxshift=3)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.SIGMA)
    rc, out, rej, _, err = _with_budget(N * C * W * 2 - 1, lambda c: c.stack_host(desc, frames) + (c.error(),))
    assert rc == -2 and "fit" in err


@pytest.mark.parametrize("max_thread", [1, 2])
def test_host_pull_band_inherits_stale_state(gpu_ctx, max_thread):
    """host-pull row bands whose first pixel breaks early in its first pass and inherits the
    stale rejected[] of the pixel one memory row above the band (src/stacking/stacking.c:1684):
    the band is retried narrower with rows above it resident, the result equals the oracle"""
    world, H, W, N = 2, 12, 70, 6
    frames = _early_break_frames(world, H, W, N)
    z = np.zeros(N, np.int32)
    sig = (1.0, 1.0)
    ref, rej_ref = _oracle(frames, sg.MEAN, sg.SIGMA, sig, z, z, max_thread)
    b, e = sd.row_band(0, world, H)
    budget = N * W * 2 * (e - b)            # bands of exactly the planted band's rows
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMA, sig=sig, shiftx=z, shifty=z,
                              max_thread=max_thread, max_number_of_rows=H)
    rc, out, rej, _, err = _with_budget(budget, lambda c: c.stack_host(desc, frames) + (c.error(),))
    assert rc == 0, err
    assert_same(out, ref, f"host bands with stale state, thr={max_thread}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)


@pytest.mark.parametrize("method,rejection", CASES + [(sg.SUM, sg.NO_REJEC)])
@pytest.mark.parametrize("devs,band_rows", [([0, 0], 0), ([0, 0, 0], 4), ([0, 0, 0, 0, 0], 0)])
def test_host_pull_device_slots(gpu_ctx, method, rejection, devs, band_rows):
    """sg_stack_u16 on a context of several device slots (here all on one card): each slot takes
    a contiguous share of the output rows, pulls its frame rows with its own readers and stacks
    them (banded under a budget when band_rows > 0); SUM scales by the maximum over every slot.
    Equal to the one-image oracle, counters summed"""
    N, C, H, W = 20, 2, 31, 90
    frames = orc.synth(N, C, H, W, seed=52, maxshift=5)
    sx, sy = orc.synth_shifts(N, seed=52, maxshift=5)
    sig = REJ[rejection]
    if method == sg.SUM:
        rc, ref, mref = orc.stack_sum(frames, sx, sy)
        assert rc == 0 and mref > 65535
        rej_ref = np.zeros((3, 2), np.uint64)
    else:
        ref, rej_ref = _oracle(frames, method, rejection, sig, sx, sy, 4)
    desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=4, max_number_of_rows=H)
    if band_rows:
        halo = 0 if method == sg.MEDIAN else int(sy.max() - sy.min())
        budget = N * C * W * 2 * (band_rows + halo)
        rc, out, rej, maxim, err = _with_budget(budget, lambda c: c.stack_host(desc, frames) + (c.error(),), devs)
    else:
        with sg.Context(devs) as c:
            rc, out, rej, maxim = c.stack_host(desc, frames)
            err = c.error()
    assert rc == 0, err
    assert_same(out, ref, f"slots={len(devs)} method={method} rej={rejection} rows={band_rows}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    if method == sg.SUM:
        assert maxim == mref


@pytest.mark.parametrize("devs", [None, [0, 0]])
def test_host_pull_cancel(gpu_ctx, devs):
    """the caller's get_thread_run() turning false mid-read: the call stops and returns -1
    (stacking.c:1539), whichever slot's reader polls it"""
    N, C, H, W = 12, 1, 24, 64
    frames = orc.synth(N, C, H, W, seed=3, maxshift=3)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=sg.SIGMA)
    with sg.Context(devs) as c:
        rc, out, rej, _ = c.stack_host(desc, frames, cancel_after=5)
        assert rc == -1
        rc, out, rej, _ = c.stack_host(desc, frames)       # the context stays usable
        assert rc == 0, c.error()


@pytest.mark.parametrize("flags", [0, sg.RESULT_AT_COLLECT])
@pytest.mark.parametrize("method,rejection", [(sg.MEAN, sg.SIGMA), (sg.MEAN, sg.WINSORIZED),
                                              (sg.MEAN, sg.PERCENTILE), (sg.MEDIAN, sg.NO_REJEC),
                                              (sg.MEAN, sg.NO_REJEC), (sg.MEAN, sg.LINEARFIT),
                                              (sg.MEAN, sg.SIGMEDIAN)])
def test_async_bands_collect(gpu_ctx, method, rejection, flags):
    """sg_stack_u16_device_async: every band queued without waiting (more calls than the two
    counter slots, so earlier calls are folded on the way), then sg_stack_collect: the image and
    the SUMMED rejection counters equal the oracle's; with SG_STACK_RESULT_AT_COLLECT each call's
    redo / replay / counter work runs on the tail stream beside the next band's main kernel"""
    import torch
    N, C, H, W = 40, 2, 48, 200
    frames = orc.synth(N, C, H, W, seed=61, maxshift=5)
    sx, sy = orc.synth_shifts(N, seed=61, maxshift=5)
    sig = REJ[rejection]
    ref, rej_ref = _oracle(frames, method, rejection, sig, sx, sy, 4)
    d_out = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    full = _dev(frames)
    desc, keep = sg.make_desc(method, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=4,
                              max_number_of_rows=H, flags=flags)
    world = 5
    for r in range(world):
        b, e = sd.row_band(r, world, H)
        gpu_ctx.stack_device_async(desc, full.data_ptr(), C * H * W, H * W, d_out.data_ptr(), b, e)
    rc, rej, _ = gpu_ctx.collect()
    assert rc == 0, gpu_ctx.error()
    out = d_out.cpu().numpy().view(np.uint16).reshape(C, H, W)
    assert_same(out, ref, f"async bands method={method} rej={rejection}")
    assert np.array_equal(rej, rej_ref), (rej, rej_ref)
    rc, rej2, _ = gpu_ctx.collect()             # nothing pending: zeros
    assert rc == 0 and not rej2.any()


@pytest.mark.parametrize("rejection,sig", [(sg.SIGMA, (0.2, 0.2)), (sg.WINSORIZED, (0.3, 0.3)),
                                           (sg.SIGMA, (4.0, 3.0))])
def test_async_tail_frames_refilled(gpu_ctx, rejection, sig):
    """a band loop that REFILLS its frame buffer between two SG_STACK_RESULT_AT_COLLECT calls on
    one stream: the first call's tail kernels (redo list, replay, literal early breaks,
    which strong rejection at N = 16 produces on most pixels) still read the buffer after the
    stream has moved on, so the refill is queued behind sg_stack_wait_tail; each call's image
    equals the oracle of ITS frames and the collected counters are their sum"""
    import torch
    N, C, H, W = 16, 1, 40, 160
    fa = orc.synth(N, C, H, W, seed=71, maxshift=4)
    fb = orc.synth(N, C, H, W, seed=72, maxshift=4)
    sx, sy = orc.synth_shifts(N, seed=71, maxshift=4)
    refa, rja = _oracle(fa, sg.MEAN, rejection, sig, sx, sy, 4)
    refb, rjb = _oracle(fb, sg.MEAN, rejection, sig, sx, sy, 4)
    buf, src_b = _dev(fa), _dev(fb)
    outa = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    outb = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    # an explicit stream: handle 0 (torch's default stream) would mean the library's own stream
    s = torch.cuda.Stream()
    stream = s.cuda_stream
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                              max_thread=4, max_number_of_rows=H, flags=sg.RESULT_AT_COLLECT)
    with torch.cuda.stream(s):
        gpu_ctx.stack_device_async(desc, buf.data_ptr(), C * H * W, H * W, outa.data_ptr(), 0, H, stream=stream)
        gpu_ctx.wait_tail(stream)
        buf.copy_(src_b)            # queued on s, behind the first call's tail kernels
        gpu_ctx.stack_device_async(desc, buf.data_ptr(), C * H * W, H * W, outb.data_ptr(), 0, H, stream=stream)
    rc, rej, _ = gpu_ctx.collect()
    assert rc == 0, gpu_ctx.error()
    st = gpu_ctx.stats()
    assert_same(outa.cpu().numpy().view(np.uint16).reshape(C, H, W), refa, "first call (frames A)")
    assert_same(outb.cpu().numpy().view(np.uint16).reshape(C, H, W), refb, "second call (frames B, refilled)")
    assert np.array_equal(rej, rja + rjb), (rej, rja, rjb)
    if sig[0] < 1:
        assert st.chain_pixels + st.slow_pixels > 0, "no tail work: the test would not exercise the ordering"


def test_async_fault_reported_by_collect(gpu_ctx):
    """a refused regime met by a queued call (here SIGMEDIAN's never-ending loop) surfaces at
    sg_stack_collect, and the next collect starts clean"""
    import torch
    N, H, W = 4, 8, 16
    frames = np.full((N, 1, H, W), 1000, dtype=np.uint16)
    frames[:, 0, 3, 5] = [990, 0, 0, 1049]
    d_out = torch.zeros(H * W, dtype=torch.int16, device="cuda")
    full = _dev(frames)
    desc, keep = sg.make_desc(sg.MEAN, N, W, H, 1, rejection=sg.SIGMEDIAN, sig=(2.5, 0.7), max_thread=1,
                              max_number_of_rows=H)
    for b, e in [(0, 3), (3, 6), (6, 8)]:
        gpu_ctx.stack_device_async(desc, full.data_ptr(), H * W, H * W, d_out.data_ptr(), b, e)
    rc, _, _ = gpu_ctx.collect()
    assert rc != 0 and "never ends" in gpu_ctx.error()
    frames[:, 0, 3, 5] = 1000
    full = _dev(frames)
    gpu_ctx.stack_device_async(desc, full.data_ptr(), H * W, H * W, d_out.data_ptr(), 0, H)
    rc, _, _ = gpu_ctx.collect()
    assert rc == 0, gpu_ctx.error()
