"""ctypes binding of the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline, never by the product path.
Parity unpinned: see oracle/oracle.h.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")

_lib = None
P = ctypes.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)

    class Seq(ctypes.Structure):
        _fields_ = [("N", ctypes.c_int), ("W", ctypes.c_int), ("H", ctypes.c_int), ("C", ctypes.c_int),
                    ("frames", P)]
    lib.Seq = Seq
    lib.or_stack_mean_with_rejection.argtypes = [ctypes.POINTER(Seq), ctypes.c_int, ctypes.c_int, P, P, P,
                                                 P, P, P, ctypes.c_int, ctypes.c_int, P, P]
    lib.or_stack_mean_with_rejection_rows.argtypes = [ctypes.POINTER(Seq), ctypes.c_int, ctypes.c_int, P, P, P,
                                                      P, P, P, ctypes.c_int, ctypes.c_int, P, P, P]
    lib.or_stack_median.argtypes = [ctypes.POINTER(Seq), ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_int, P]
    lib.or_stack_summing.argtypes = [ctypes.POINTER(Seq), P, P, P, P]
    lib.or_stack_addmax.argtypes = [ctypes.POINTER(Seq), P, P, P]
    lib.or_stack_addmin.argtypes = [ctypes.POINTER(Seq), P, P, P]
    lib.or_gsl_sd_u16.argtypes = [P, ctypes.c_size_t]
    lib.or_gsl_sd_u16.restype = ctypes.c_double
    lib.or_gsl_mean_u16.argtypes = [P, ctypes.c_size_t]
    lib.or_gsl_mean_u16.restype = ctypes.c_double
    lib.or_round_to_WORD.argtypes = [ctypes.c_double]
    lib.or_round_to_WORD.restype = ctypes.c_uint16
    lib.or_synth_fill.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
    lib.or_synth_shift.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    lib.or_register_shift_dft.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P]
    lib.or_quality_estimate.argtypes = [P, ctypes.c_int, ctypes.c_int]
    lib.or_quality_estimate.restype = ctypes.c_double
    lib.or_compute_normalization.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P]
    lib.or_statistics_ikss.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
    lib.or_statistics_ikss.restype = ctypes.c_int
    lib.or_synth_window.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
    lib.or_xcorr_at.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.or_xcorr_at.restype = ctypes.c_longlong
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(P) if a is not None else None


def _arr(a, dt):
    return None if a is None else np.ascontiguousarray(a, dtype=dt)


def _seq(frames):
    lib = load()
    N, C, H, W = frames.shape
    return lib.Seq(N, W, H, C, frames.ctypes.data_as(P))


def stack_rejection(frames, rejection, sig=(4.0, 3.0), shiftx=None, shifty=None, normalize=0,
                    offset=None, mul=None, scale=None, max_thread=8, max_number_of_rows=0, row_counters=False):
    """(rc, image [C][H][W], rejection counters [3][2]); row_counters=True adds each memory row's
    low / high counts [C][H][2] (a row band's counters are their sum)"""
    lib = load()
    frames = np.ascontiguousarray(frames, dtype=np.uint16)
    N, C, H, W = frames.shape
    if max_number_of_rows <= 0:
        max_number_of_rows = H
    sx, sy = _arr(shiftx, np.int32), _arr(shifty, np.int32)
    of, mu, sc = _arr(offset, np.float64), _arr(mul, np.float64), _arr(scale, np.float64)
    sg = np.array(sig, dtype=np.float64)
    out = np.zeros((C, H, W), dtype=np.uint16)
    rej = np.zeros((3, 2), dtype=np.uint64)
    seq = _seq(frames)
    if row_counters:
        rows = np.zeros((C, H, 2), dtype=np.uint64)
        rc = lib.or_stack_mean_with_rejection_rows(ctypes.byref(seq), rejection, normalize, _p(sg), _p(sx), _p(sy),
                                                   _p(of), _p(mu), _p(sc), max_thread, max_number_of_rows,
                                                   _p(out), _p(rej), _p(rows))
        return rc, out, rej, rows
    rc = lib.or_stack_mean_with_rejection(ctypes.byref(seq), rejection, normalize, _p(sg), _p(sx), _p(sy),
                                          _p(of), _p(mu), _p(sc), max_thread, max_number_of_rows,
                                          _p(out), _p(rej))
    return rc, out, rej


def stack_median(frames, normalize=0, offset=None, mul=None, scale=None, max_thread=8, max_number_of_rows=0):
    lib = load()
    frames = np.ascontiguousarray(frames, dtype=np.uint16)
    N, C, H, W = frames.shape
    if max_number_of_rows <= 0:
        max_number_of_rows = H
    of, mu, sc = _arr(offset, np.float64), _arr(mul, np.float64), _arr(scale, np.float64)
    out = np.zeros((C, H, W), dtype=np.uint16)
    seq = _seq(frames)
    rc = lib.or_stack_median(ctypes.byref(seq), normalize, _p(of), _p(mu), _p(sc), max_thread,
                             max_number_of_rows, _p(out))
    return rc, out


def stack_sum(frames, shiftx=None, shifty=None):
    lib = load()
    frames = np.ascontiguousarray(frames, dtype=np.uint16)
    N, C, H, W = frames.shape
    sx, sy = _arr(shiftx, np.int32), _arr(shifty, np.int32)
    out = np.zeros((C, H, W), dtype=np.uint16)
    mx = np.zeros(1, dtype=np.uint64)
    seq = _seq(frames)
    rc = lib.or_stack_summing(ctypes.byref(seq), _p(sx), _p(sy), _p(out), _p(mx))
    return rc, out, int(mx[0])


def stack_maxmin(frames, is_max, shiftx=None, shifty=None):
    lib = load()
    frames = np.ascontiguousarray(frames, dtype=np.uint16)
    N, C, H, W = frames.shape
    sx, sy = _arr(shiftx, np.int32), _arr(shifty, np.int32)
    out = np.zeros((C, H, W), dtype=np.uint16)
    seq = _seq(frames)
    f = lib.or_stack_addmax if is_max else lib.or_stack_addmin
    rc = f(ctypes.byref(seq), _p(sx), _p(sy), _p(out))
    return rc, out


def synth(nframes, C, H, W, seed=1, maxshift=16, row_begin=0, row_end=None):
    lib = load()
    if row_end is None:
        row_end = H
    frames = np.zeros((nframes, C, H, W), dtype=np.uint16)
    lib.or_synth_fill(_p(frames), nframes, C, H, W, row_begin, row_end, seed, maxshift)
    return frames


def synth_window(nframes, c, y0, x0, h, w, seed=1, maxshift=16):
    """channel c, memory rows [y0, y0+h), columns [x0, x0+w) of every synthetic frame: [N][h][w]"""
    lib = load()
    out = np.zeros((nframes, h, w), dtype=np.uint16)
    lib.or_synth_window(_p(out), nframes, c, y0, x0, h, w, seed, maxshift)
    return out


def xcorr_at(ref, img, ky, kx):
    """exact sum_n ref(n + k) img(n) (circular) at k = (ky, kx): the integer behind the
    reference's correlation-plane entry (divided by S^2)"""
    lib = load()
    ref = np.ascontiguousarray(ref, dtype=np.uint16)
    img = np.ascontiguousarray(img, dtype=np.uint16)
    return int(lib.or_xcorr_at(_p(ref), _p(img), ref.shape[0], ky % ref.shape[0], kx % ref.shape[0]))


def synth_shifts(nframes, seed=1, maxshift=16):
    """(shiftx, shifty) that re-align the synthetic frames: (-dx_f, -dy_f)."""
    lib = load()
    sx = np.zeros(nframes, dtype=np.int32)
    sy = np.zeros(nframes, dtype=np.int32)
    for f in range(nframes):
        dx, dy = ctypes.c_int(), ctypes.c_int()
        lib.or_synth_shift(seed, f, maxshift, ctypes.byref(dx), ctypes.byref(dy))
        sx[f], sy[f] = -dx.value, -dy.value
    return sx, sy


def gsl_sd(data):
    lib = load()
    d = np.ascontiguousarray(data, dtype=np.uint16)
    return lib.or_gsl_sd_u16(_p(d), len(d))


def gsl_mean(data):
    lib = load()
    d = np.ascontiguousarray(data, dtype=np.uint16)
    return lib.or_gsl_mean_u16(_p(d), len(d))


def register_dft(sel, ref_image=0, included=None):
    lib = load()
    sel = np.ascontiguousarray(sel, dtype=np.uint16)
    n, S, _ = sel.shape
    inc = _arr(included, np.int32)
    sx = np.zeros(n, dtype=np.int32)
    sy = np.zeros(n, dtype=np.int32)
    q = np.zeros(n, dtype=np.float64)
    lib.or_register_shift_dft(_p(sel), n, S, ref_image, _p(inc), _p(sx), _p(sy), _p(q))
    return sx, sy, q


def quality(img):
    lib = load()
    img = np.ascontiguousarray(img, dtype=np.uint16)
    h, w = img.shape
    return lib.or_quality_estimate(_p(img), w, h)


def compute_normalization(mode, location, scalev, ref_image=0):
    lib = load()
    n = len(location)
    loc = np.ascontiguousarray(location, dtype=np.float64)
    sc = np.ascontiguousarray(scalev, dtype=np.float64)
    off, mul, scale = np.zeros(n), np.ones(n), np.ones(n)
    lib.or_compute_normalization(n, ref_image, mode, _p(loc), _p(sc), _p(off), _p(mul), _p(scale))
    return off, mul, scale


def statistics_ikss(frame):
    """frame [C][H][W] u16 -> (rc, location, scale) of layer 0 (statistics.c IKSS)"""
    lib = load()
    f = np.ascontiguousarray(frame, dtype=np.uint16)
    C, H, W = f.shape
    loc = ctypes.c_double(0.0)
    sc = ctypes.c_double(0.0)
    rc = lib.or_statistics_ikss(_p(f), C, H, W, ctypes.byref(loc), ctypes.byref(sc))
    return rc, loc.value, sc.value
