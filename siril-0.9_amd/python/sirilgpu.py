"""ctypes binding of libsirilgpu.so (include/sirilgpu.h) for tests, bench.py and smoke().

The product is the C ABI + gfx950 kernels; this module only marshals arguments.  It
refuses to run if the shared library has not been built: there is no Python or CPU
fallback for any pixel.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("SG_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libsirilgpu.so")  # A/B builds

# enum values (src/stacking/stacking.c:54-56, src/stacking/stacking.h:14-30)
SUM, MEAN, MEDIAN, MAX, MIN = range(5)
NO_REJEC, PERCENTILE, SIGMA, SIGMEDIAN, WINSORIZED, LINEARFIT = range(6)
NO_NORM, ADDITIVE, MULTIPLICATIVE, ADDITIVE_SCALING, MULTIPLICATIVE_SCALING = range(5)
PATH_AUTO, PATH_SORTED = 0, 1
RESULT_AT_COLLECT = 1        # sg_stack_desc.flags (SG_STACK_RESULT_AT_COLLECT)

SG_OK = 0
SG_ERR_GENERIC, SG_ERR_SIZE, SG_ERR_READ, SG_ERR_DEVICE = -1, -2, -3, -10


class StackDesc(ctypes.Structure):
    _fields_ = [
        ("method", ctypes.c_int),
        ("rejection", ctypes.c_int),
        ("normalize", ctypes.c_int),
        ("sig", ctypes.c_double * 2),
        ("nb_frames", ctypes.c_int),
        ("width", ctypes.c_int),
        ("height", ctypes.c_int),
        ("nb_layers", ctypes.c_int),
        ("shiftx", ctypes.POINTER(ctypes.c_int)),
        ("shifty", ctypes.POINTER(ctypes.c_int)),
        ("offset", ctypes.POINTER(ctypes.c_double)),
        ("mul", ctypes.POINTER(ctypes.c_double)),
        ("scale", ctypes.POINTER(ctypes.c_double)),
        ("max_thread", ctypes.c_int),
        ("max_number_of_rows", ctypes.c_int),
        ("kernel_path", ctypes.c_int),
        ("resident_rows", ctypes.c_int * 2),
        ("flags", ctypes.c_int),
        ("reserved", ctypes.c_int * 2),
    ]


class StackStats(ctypes.Structure):
    _fields_ = [
        ("kernel_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("slow_pixels", ctypes.c_uint64),
        ("chain_pixels", ctypes.c_uint64),
        ("launches", ctypes.c_uint64),
        ("main_kernel_blocks", ctypes.c_int),
        ("path", ctypes.c_int),
        ("reg_ties_resolved", ctypes.c_uint64),
        ("reg_ties_unresolved", ctypes.c_uint64),
        ("reg_fp64_reruns", ctypes.c_uint64),
        ("compact_pixels", ctypes.c_uint64),
        ("reg_ms", ctypes.c_double),
        ("exported_pixels", ctypes.c_uint64),
        ("norm_fma", ctypes.c_int64),
    ]


class Rect(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int), ("y", ctypes.c_int), ("w", ctypes.c_int), ("h", ctypes.c_int)]


READ_REGION_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(Rect))
CONT_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)

class SeqInfo(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("nb_layers", ctypes.c_int),
                ("nb_frames", ctypes.c_int), ("bytes_per_sample", ctypes.c_int), ("source", ctypes.c_int),
                ("ser_color_id", ctypes.c_int), ("frame_bytes", ctypes.c_int64)]


# every symbol include/sirilgpu.h and include/sirilgpu_io.h declare
EXPORTS = ["sg_init", "sg_shutdown", "sg_last_error", "sg_stack_u16", "sg_stack_u16_device",
           "sg_stack_u16_device_async", "sg_stack_collect", "sg_stack_wait_tail", "sg_device_count",
           "sg_get_last_stats", "sg_register_dft_u16", "sg_register_dft_u16_device",
           "sg_register_dft_u16_device_raw", "sg_register_dft_u16_device_pitched", "sg_synth_fill_device",
           "sg_seq_open_ser", "sg_seq_open_fits", "sg_seq_close", "sg_seq_get_info", "sg_seq_read_region",
           "sg_seq_read_frame", "sg_seq_load_device", "sg_seq_set_debayer", "sg_warp_u16", "sg_warp_u16_device",
           "sg_frame_stats_ikss_device", "sg_compute_normalization", "sg_seqfile_read", "sg_seqfile_create",
           "sg_seqfile_free", "sg_seqfile_get_info", "sg_seqfile_get_images", "sg_seqfile_set_image",
           "sg_seqfile_get_registration", "sg_seqfile_set_registration", "sg_seqfile_write"]
# opencv_interpolation (src/core/siril.h:257-264)
OPENCV_NEAREST, OPENCV_LINEAR, OPENCV_AREA, OPENCV_CUBIC, OPENCV_LANCZOS4 = range(5)

_lib = None


def load():
    """Load libsirilgpu.so; raises if it is missing (fail loudly, no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `make -C siril-0.9_amd` (no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.c_void_p
    lib.sg_init.argtypes = [ctypes.POINTER(P), ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    lib.sg_init.restype = ctypes.c_int
    lib.sg_shutdown.argtypes = [P]
    lib.sg_shutdown.restype = None
    lib.sg_last_error.argtypes = [P]
    lib.sg_last_error.restype = ctypes.c_char_p
    lib.sg_stack_u16.argtypes = [P, ctypes.POINTER(StackDesc), READ_REGION_FN, P, CONT_FN, P,
                                 ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64)]
    lib.sg_stack_u16.restype = ctypes.c_int
    lib.sg_stack_u16_device.argtypes = [P, ctypes.c_int, ctypes.POINTER(StackDesc), P, ctypes.c_int64,
                                        ctypes.c_int64, P, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), P]
    lib.sg_stack_u16_device.restype = ctypes.c_int
    lib.sg_stack_u16_device_async.argtypes = [P, ctypes.c_int, ctypes.POINTER(StackDesc), P, ctypes.c_int64,
                                              ctypes.c_int64, P, ctypes.c_int, ctypes.c_int, P]
    lib.sg_stack_u16_device_async.restype = ctypes.c_int
    lib.sg_stack_collect.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.sg_stack_collect.restype = ctypes.c_int
    lib.sg_stack_wait_tail.argtypes = [P, ctypes.c_int, ctypes.c_void_p]
    lib.sg_stack_wait_tail.restype = ctypes.c_int
    lib.sg_device_count.argtypes = [P, ctypes.POINTER(ctypes.c_int)]
    lib.sg_device_count.restype = ctypes.c_int
    lib.sg_get_last_stats.argtypes = [P, ctypes.POINTER(StackStats)]
    lib.sg_get_last_stats.restype = ctypes.c_int
    lib.sg_synth_fill_device.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                         ctypes.c_int, ctypes.c_int64, P]
    lib.sg_synth_fill_device.restype = ctypes.c_int
    lib.sg_synth_fill_frames_device.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_uint64, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, P]
    lib.sg_synth_fill_frames_device.restype = ctypes.c_int
    lib.sg_register_dft_u16.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P]
    lib.sg_register_dft_u16.restype = ctypes.c_int
    lib.sg_register_dft_u16_device.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               P, P, P, P, P]
    lib.sg_register_dft_u16_device.restype = ctypes.c_int
    lib.sg_register_dft_u16_device_raw.argtypes = lib.sg_register_dft_u16_device.argtypes
    lib.sg_register_dft_u16_device_raw.restype = ctypes.c_int
    lib.sg_register_dft_u16_device_pitched.argtypes = [P, ctypes.c_int, P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                                       ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int, P]
    lib.sg_register_dft_u16_device_pitched.restype = ctypes.c_int
    lib.sg_seq_open_ser.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
    lib.sg_seq_open_ser.restype = ctypes.c_int
    lib.sg_seq_open_fits.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.POINTER(P)]
    lib.sg_seq_open_fits.restype = ctypes.c_int
    lib.sg_seq_close.argtypes = [P]
    lib.sg_seq_close.restype = None
    lib.sg_seq_get_info.argtypes = [P, ctypes.POINTER(SeqInfo)]
    lib.sg_seq_get_info.restype = ctypes.c_int
    lib.sg_seq_read_region.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint16),
                                       ctypes.POINTER(Rect)]
    lib.sg_seq_read_region.restype = ctypes.c_int
    lib.sg_seq_read_frame.argtypes = [P, ctypes.c_int, ctypes.POINTER(ctypes.c_uint16)]
    lib.sg_seq_read_frame.restype = ctypes.c_int
    lib.sg_seq_read_selection.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Rect),
                                          ctypes.POINTER(ctypes.c_uint16)]
    lib.sg_seq_read_selection.restype = ctypes.c_int
    lib.sg_frame_stats_ikss.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P]
    lib.sg_frame_stats_ikss.restype = ctypes.c_int
    lib.sg_seq_load_device.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, ctypes.c_int64, P]
    lib.sg_seq_load_device.restype = ctypes.c_int
    lib.sg_frame_stats_ikss_device.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int64, P, P, P]
    lib.sg_frame_stats_ikss_device.restype = ctypes.c_int
    lib.sg_compute_normalization.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P]
    lib.sg_compute_normalization.restype = ctypes.c_int
    lib.sg_seqfile_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
    lib.sg_seqfile_create.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.POINTER(P)]
    lib.sg_seqfile_free.argtypes = [P]
    lib.sg_seqfile_free.restype = None
    lib.sg_seqfile_get_info.argtypes = [P, ctypes.POINTER(SeqFileInfo)]
    lib.sg_seqfile_get_images.argtypes = [P, P, P, P, P]
    lib.sg_seqfile_set_image.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
    lib.sg_seqfile_get_registration.argtypes = [P, ctypes.c_int, P, P, P, P, P, P, P]
    lib.sg_seqfile_set_registration.argtypes = [P, ctypes.c_int, P, P, P]
    lib.sg_seqfile_write.argtypes = [P, ctypes.c_char_p]
    lib.sg_seq_set_debayer.argtypes = [P, ctypes.c_int]
    lib.sg_seq_set_debayer.restype = ctypes.c_int
    lib.sg_warp_u16.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    lib.sg_warp_u16.restype = ctypes.c_int
    lib.sg_warp_u16_device.argtypes = [P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int, P]
    lib.sg_warp_u16_device.restype = ctypes.c_int
    _lib = lib
    return lib


class SeqFileInfo(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 512), ("beg", ctypes.c_int), ("number", ctypes.c_int),
                ("selnum", ctypes.c_int), ("fixed", ctypes.c_int), ("reference_image", ctypes.c_int),
                ("type", ctypes.c_int), ("nb_layers", ctypes.c_int)]


SEQFILE_REGULAR, SEQFILE_SER, SEQFILE_FILM = 0, 1, 2


class SeqFile:
    """A Siril .seq file (include/sirilgpu_io.h sg_seqfile_*): host-only."""

    def __init__(self, handle):
        self.lib = load()
        self.h = handle

    @classmethod
    def read(cls, path):
        lib = load()
        h = ctypes.c_void_p()
        rc = lib.sg_seqfile_read(os.fsencode(path), ctypes.byref(h))
        if rc != SG_OK:
            raise OSError(f"sg_seqfile_read({path}) failed ({rc})")
        return cls(h)

    @classmethod
    def create(cls, name, number, beg=1, fixed=5, reference_image=-1, type=SEQFILE_REGULAR, nb_layers=1):
        lib = load()
        h = ctypes.c_void_p()
        rc = lib.sg_seqfile_create(name.encode(), beg, number, fixed, reference_image, type, nb_layers, ctypes.byref(h))
        if rc != SG_OK:
            raise RuntimeError(f"sg_seqfile_create failed ({rc})")
        return cls(h)

    def close(self):
        if self.h:
            self.lib.sg_seqfile_free(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def info(self):
        i = SeqFileInfo()
        self.lib.sg_seqfile_get_info(self.h, ctypes.byref(i))
        return i

    def images(self):
        n = self.info().number
        fn, inc, hs = (np.zeros(n, np.int32) for _ in range(3))
        st = np.zeros((n, 10), np.float64)
        self.lib.sg_seqfile_get_images(self.h, fn.ctypes.data_as(ctypes.c_void_p), inc.ctypes.data_as(ctypes.c_void_p),
                                       hs.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p))
        return fn, inc, hs, st

    def set_image(self, index, filenum, incl, stats=None):
        st = None if stats is None else np.ascontiguousarray(stats, dtype=np.float64)
        rc = self.lib.sg_seqfile_set_image(self.h, index, filenum, incl,
                                           None if st is None else st.ctypes.data_as(ctypes.c_void_p))
        if rc != SG_OK:
            raise RuntimeError("sg_seqfile_set_image failed")

    def registration(self, layer):
        """(rc, shiftx, shifty, rot_centre_x, rot_centre_y, angle, fwhm, quality); rc 1 = no data"""
        n = self.info().number
        sx, sy = np.zeros(n, np.int32), np.zeros(n, np.int32)
        fl = [np.zeros(n, np.float32) for _ in range(4)]
        q = np.zeros(n, np.float64)
        rc = self.lib.sg_seqfile_get_registration(self.h, layer, sx.ctypes.data_as(ctypes.c_void_p),
                                                  sy.ctypes.data_as(ctypes.c_void_p),
                                                  *[a.ctypes.data_as(ctypes.c_void_p) for a in fl],
                                                  q.ctypes.data_as(ctypes.c_void_p))
        return (rc, sx, sy, *fl, q)

    def set_registration(self, layer, shiftx, shifty, quality=None):
        sx = np.ascontiguousarray(shiftx, dtype=np.int32)
        sy = np.ascontiguousarray(shifty, dtype=np.int32)
        q = None if quality is None else np.ascontiguousarray(quality, dtype=np.float64)
        rc = self.lib.sg_seqfile_set_registration(self.h, layer, sx.ctypes.data_as(ctypes.c_void_p),
                                                  sy.ctypes.data_as(ctypes.c_void_p),
                                                  None if q is None else q.ctypes.data_as(ctypes.c_void_p))
        if rc != SG_OK:
            raise RuntimeError("sg_seqfile_set_registration failed")

    def write(self, path):
        rc = self.lib.sg_seqfile_write(self.h, os.fsencode(path))
        if rc != SG_OK:
            raise OSError(f"sg_seqfile_write({path}) failed ({rc})")


# sensor_pattern (src/core/siril.h:266-271)
BAYER_RGGB, BAYER_BGGR, BAYER_GBRG, BAYER_GRBG = 0, 1, 2, 3


class Seq:
    """An opened SER file or FITS sequence (include/sirilgpu_io.h); host-side reads need no GPU."""

    def __init__(self, handle):
        self.lib = load()
        self.h = handle
        info = SeqInfo()
        rc = self.lib.sg_seq_get_info(self.h, ctypes.byref(info))
        if rc != SG_OK:
            raise RuntimeError(f"sg_seq_get_info failed ({rc})")
        self.info = info
        self.shape = (info.nb_frames, info.nb_layers, info.height, info.width)

    @classmethod
    def open_ser(cls, path):
        lib = load()
        h = ctypes.c_void_p()
        rc = lib.sg_seq_open_ser(os.fsencode(path), ctypes.byref(h))
        if rc != SG_OK:
            raise OSError(f"sg_seq_open_ser({path}) failed ({rc})")
        return cls(h)

    @classmethod
    def open_fits(cls, paths):
        lib = load()
        arr = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
        h = ctypes.c_void_p()
        rc = lib.sg_seq_open_fits(arr, len(paths), ctypes.byref(h))
        if rc != SG_OK:
            raise OSError(f"sg_seq_open_fits failed ({rc})")
        return cls(h)

    def close(self):
        if self.h:
            self.lib.sg_seq_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_debayer(self, pattern=-1):
        """demosaic a CFA SER on device loads (bilinear); pattern BAYER_* or -1 = from the header"""
        rc = self.lib.sg_seq_set_debayer(self.h, pattern)
        if rc != SG_OK:
            raise RuntimeError(f"sg_seq_set_debayer failed ({rc})")
        info = SeqInfo()
        self.lib.sg_seq_get_info(self.h, ctypes.byref(info))
        self.info = info
        self.shape = (info.nb_frames, info.nb_layers, info.height, info.width)

    def read_region(self, layer, index, x, y, w, h):
        """top-down band (seq_opened_read_region); returns (rc, array[h][w])"""
        buf = np.zeros((h, w), dtype=np.uint16)
        rc = self.lib.sg_seq_read_region(self.h, layer, index, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)),
                                         ctypes.byref(Rect(x, y, w, h)))
        return rc, buf

    def read_selection(self, layer, index, x, y, w, h):
        """seq_read_frame_part: the selection (display coordinates) bottom-up; (rc, array[h][w])"""
        buf = np.zeros((h, w), dtype=np.uint16)
        rc = self.lib.sg_seq_read_selection(self.h, layer, index, ctypes.byref(Rect(x, y, w, h)),
                                            buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)))
        return rc, buf

    def read_frame(self, index):
        out = np.zeros(self.shape[1:], dtype=np.uint16)
        rc = self.lib.sg_seq_read_frame(self.h, index, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)))
        if rc != SG_OK:
            raise RuntimeError(f"sg_seq_read_frame({index}) failed ({rc})")
        return out


def _iptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int)) if a is not None else None


def _dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if a is not None else None


def make_desc(method, N, W, H, C, rejection=NO_REJEC, normalize=NO_NORM, sig=(4.0, 3.0),
              shiftx=None, shifty=None, offset=None, mul=None, scale=None, max_thread=8,
              max_number_of_rows=0, kernel_path=PATH_AUTO, resident_rows=None, flags=0):
    """Build a StackDesc; returns (desc, keepalive) -- keep the arrays alive during the call.
    resident_rows = (first, end) memory rows present at the device frames (None = all)."""
    keep = []

    def arr(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a

    sx, sy = arr(shiftx, np.int32), arr(shifty, np.int32)
    of, mu, sc = arr(offset, np.float64), arr(mul, np.float64), arr(scale, np.float64)
    d = StackDesc()
    d.method, d.rejection, d.normalize = method, rejection, normalize
    d.sig[0], d.sig[1] = float(sig[0]), float(sig[1])
    d.nb_frames, d.width, d.height, d.nb_layers = N, W, H, C
    d.shiftx, d.shifty = _iptr(sx), _iptr(sy)
    d.offset, d.mul, d.scale = _dptr(of), _dptr(mu), _dptr(sc)
    d.max_thread, d.max_number_of_rows = max_thread, max_number_of_rows
    d.kernel_path = kernel_path
    d.flags = flags
    if resident_rows is not None:
        d.resident_rows[0], d.resident_rows[1] = int(resident_rows[0]), int(resident_rows[1])
    return d, keep


class Context:
    def __init__(self, devices=None):
        self.lib = load()
        self.ctx = ctypes.c_void_p()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = self.lib.sg_init(ctypes.byref(self.ctx), len(devices), arr)
        else:
            rc = self.lib.sg_init(ctypes.byref(self.ctx), 0, None)
        if rc != SG_OK:
            raise RuntimeError(f"sg_init failed ({rc})")

    def close(self):
        if self.ctx:
            self.lib.sg_shutdown(self.ctx)
            self.ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def error(self):
        return self.lib.sg_last_error(self.ctx).decode()

    def check(self, rc, what):
        if rc != SG_OK:
            raise RuntimeError(f"{what} failed ({rc}): {self.error()}")

    def stats(self):
        st = StackStats()
        self.check(self.lib.sg_get_last_stats(self.ctx, ctypes.byref(st)), "sg_get_last_stats")
        return st

    def stack_device(self, desc, d_frames, frame_stride, plane_stride, d_out, row_begin, row_end,
                     stream=None, dev_index=0):
        rej = (ctypes.c_uint64 * 6)()
        maxim = ctypes.c_uint64(0)
        rc = self.lib.sg_stack_u16_device(self.ctx, dev_index, ctypes.byref(desc), ctypes.c_void_p(d_frames),
                                          frame_stride, plane_stride, ctypes.c_void_p(d_out), row_begin,
                                          row_end, rej, ctypes.byref(maxim),
                                          ctypes.c_void_p(stream) if stream else None)
        self.check(rc, "sg_stack_u16_device")
        return np.array(list(rej), dtype=np.uint64).reshape(3, 2), int(maxim.value)

    def stack_device_async(self, desc, d_frames, frame_stride, plane_stride, d_out, row_begin, row_end,
                           stream=None, dev_index=0):
        """sg_stack_u16_device_async: queued, nothing waited for; results via collect()"""
        rc = self.lib.sg_stack_u16_device_async(self.ctx, dev_index, ctypes.byref(desc), ctypes.c_void_p(d_frames),
                                                frame_stride, plane_stride, ctypes.c_void_p(d_out), row_begin,
                                                row_end, ctypes.c_void_p(stream) if stream else None)
        self.check(rc, "sg_stack_u16_device_async")

    def wait_tail(self, stream=None, dev_index=0):
        """sg_stack_wait_tail: work queued on `stream` from now on waits for the async calls' tail kernels"""
        self.check(self.lib.sg_stack_wait_tail(self.ctx, dev_index, ctypes.c_void_p(stream) if stream else None),
                   "sg_stack_wait_tail")

    def collect(self, dev_index=0):
        """sg_stack_collect: (rc, summed rejection counters [3][2], max SUM maximum) of the pending calls"""
        rej = (ctypes.c_uint64 * 6)()
        maxim = ctypes.c_uint64(0)
        rc = self.lib.sg_stack_collect(self.ctx, dev_index, rej, ctypes.byref(maxim))
        return rc, np.array(list(rej), dtype=np.uint64).reshape(3, 2), int(maxim.value)

    def device_count(self):
        n = ctypes.c_int(0)
        self.check(self.lib.sg_device_count(self.ctx, ctypes.byref(n)), "sg_device_count")
        return n.value

    def load_seq_device(self, seq, d_frames, first=0, count=None, frame_stride=0, dev_index=0, stream=None):
        """frames of an opened Seq decoded on the device (sg_seq_load_device)"""
        if count is None:
            count = seq.shape[0] - first
        rc = self.lib.sg_seq_load_device(self.ctx, dev_index, seq.h, first, count, ctypes.c_void_p(d_frames),
                                         frame_stride, ctypes.c_void_p(stream) if stream else None)
        self.check(rc, "sg_seq_load_device")

    def frame_stats_ikss(self, d_frames, nframes, C, H, W, frame_stride=0, dev_index=0, stream=None):
        """per-frame IKSS location / scale of layer 0 (sg_frame_stats_ikss_device);
        returns (rc, location[nframes], scale[nframes])"""
        loc = np.zeros(nframes, dtype=np.float64)
        scl = np.zeros(nframes, dtype=np.float64)
        rc = self.lib.sg_frame_stats_ikss_device(self.ctx, dev_index, ctypes.c_void_p(d_frames), nframes, C, H, W,
                                                 frame_stride, loc.ctypes.data_as(ctypes.c_void_p),
                                                 scl.ctypes.data_as(ctypes.c_void_p),
                                                 ctypes.c_void_p(stream) if stream else None)
        return rc, loc, scl

    def warp(self, image, hom, out_size=None, interpolation=OPENCV_LINEAR):
        """cvTransformImage on a memory-order image [C][H][W]; hom = the 3x3 homography
        (Homography h00..h22), out_size = (ref.x, ref.y)"""
        image = np.ascontiguousarray(image, dtype=np.uint16)
        C, H, W = image.shape
        oW, oH = out_size if out_size else (W, H)
        out = np.zeros((C, oH, oW), dtype=np.uint16)
        h = (ctypes.c_double * 9)(*[float(v) for v in np.asarray(hom, dtype=np.float64).reshape(9)])
        rc = self.lib.sg_warp_u16(self.ctx, image.ctypes.data_as(ctypes.c_void_p), W, H, C,
                                  out.ctypes.data_as(ctypes.c_void_p), oW, oH, h, interpolation)
        self.check(rc, "sg_warp_u16")
        return out

    def stack_seq(self, desc, seq):
        """Host-pull stack whose pull callback is the library's own sg_seq_read_region (C),
        i.e. stack_mean_with_rejection & co. reading the sequence's files directly."""
        N, C, H, W = seq.shape
        rf = ctypes.cast(self.lib.sg_seq_read_region, READ_REGION_FN)
        cf = CONT_FN(lambda user: 1)
        out = np.zeros((C, H, W), dtype=np.uint16)
        rej = (ctypes.c_uint64 * 6)()
        maxim = ctypes.c_uint64(0)
        rc = self.lib.sg_stack_u16(self.ctx, ctypes.byref(desc), rf, seq.h, cf, None,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), rej,
                                   ctypes.byref(maxim))
        return rc, out, np.array(list(rej), dtype=np.uint64).reshape(3, 2), int(maxim.value)

    def stack_host(self, desc, frames, cancel_after=None):
        """Host-pull path: frames[N][C][H][W] (memory order) served through a
        seq_opened_read_region-shaped callback returning top-down bands."""
        N, C, H, W = frames.shape
        calls = [0]

        def read_region(user, layer, index, buf, area):
            a = area.contents
            band = frames[index, layer, H - 1 - (a.y + np.arange(a.h)), a.x:a.x + a.w]
            dst = np.ctypeslib.as_array(buf, shape=(a.h * a.w,))
            dst[:] = np.ascontiguousarray(band).reshape(-1)
            return 0

        def cont(user):
            calls[0] += 1
            return 0 if (cancel_after is not None and calls[0] > cancel_after) else 1

        rf, cf = READ_REGION_FN(read_region), CONT_FN(cont)
        out = np.zeros((C, H, W), dtype=np.uint16)
        rej = (ctypes.c_uint64 * 6)()
        maxim = ctypes.c_uint64(0)
        rc = self.lib.sg_stack_u16(self.ctx, ctypes.byref(desc), rf, None, cf, None,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), rej,
                                   ctypes.byref(maxim))
        return rc, out, np.array(list(rej), dtype=np.uint64).reshape(3, 2), int(maxim.value)

    def register_dft(self, sel, ref_image=0, included=None):
        """register_shift_dft on host selections sel[nframes][S][S] (bottom-up, one layer)."""
        sel = np.ascontiguousarray(sel, dtype=np.uint16)
        n, S, S2 = sel.shape
        assert S == S2
        inc = None if included is None else np.ascontiguousarray(included, dtype=np.int32)
        sx = np.zeros(n, dtype=np.int32)
        sy = np.zeros(n, dtype=np.int32)
        q = np.zeros(n, dtype=np.float64)
        P = ctypes.c_void_p
        rc = self.lib.sg_register_dft_u16(self.ctx, sel.ctypes.data_as(P), n, S, ref_image,
                                          inc.ctypes.data_as(P) if inc is not None else None,
                                          sx.ctypes.data_as(P), sy.ctypes.data_as(P), q.ctypes.data_as(P))
        self.check(rc, "sg_register_dft_u16")
        return sx, sy, q

    def register_dft_device(self, d_sel, nframes, S, ref_image=0, included=None, stream=None, dev_index=0,
                            raw_quality=False, frame_pitch=0, row_pitch=0):
        """register_shift_dft on device selections; raw_quality: the shard entry point
        (sg_register_dft_u16_device_raw: QualityEstimate values, not normalised); frame_pitch /
        row_pitch (elements): selections read in place from resident frames
        (sg_register_dft_u16_device_pitched)"""
        inc = None if included is None else np.ascontiguousarray(included, dtype=np.int32)
        sx = np.zeros(nframes, dtype=np.int32)
        sy = np.zeros(nframes, dtype=np.int32)
        q = np.zeros(nframes, dtype=np.float64)
        P = ctypes.c_void_p
        args = (inc.ctypes.data_as(P) if inc is not None else None, sx.ctypes.data_as(P), sy.ctypes.data_as(P),
                q.ctypes.data_as(P))
        if frame_pitch or row_pitch:
            rc = self.lib.sg_register_dft_u16_device_pitched(
                self.ctx, dev_index, P(d_sel), frame_pitch or S * S, row_pitch or S, nframes, S, ref_image, *args,
                1 if raw_quality else 0, P(stream) if stream else None)
            self.check(rc, "sg_register_dft_u16_device_pitched")
            return sx, sy, q
        fn = self.lib.sg_register_dft_u16_device_raw if raw_quality else self.lib.sg_register_dft_u16_device
        rc = fn(self.ctx, dev_index, P(d_sel), nframes, S, ref_image, *args, P(stream) if stream else None)
        self.check(rc, "sg_register_dft_u16_device" + ("_raw" if raw_quality else ""))
        return sx, sy, q

    def synth_fill(self, d_frames, nframes, C, H, W, row_begin, row_end, seed, maxshift, dev_index=0,
                   frame_stride=0, first_frame=0, plane_stride=0):
        rc = self.lib.sg_synth_fill_frames_device(self.ctx, dev_index, ctypes.c_void_p(d_frames), first_frame, nframes,
                                                  C, H, W, row_begin, row_end, seed, maxshift, frame_stride,
                                                  plane_stride, None)
        self.check(rc, "sg_synth_fill_frames_device")


def compute_normalization(mode, location, scale, ref_image=0):
    """compute_normalization (stacking.c:125-190) through the C ABI: (offset, mul, scale)"""
    lib = load()
    n = len(location)
    loc = np.ascontiguousarray(location, dtype=np.float64)
    sc = np.ascontiguousarray(scale, dtype=np.float64)
    off, mul, so = (np.zeros(n), np.zeros(n), np.zeros(n))
    rc = lib.sg_compute_normalization(mode, n, ref_image, loc.ctypes.data_as(ctypes.c_void_p),
                                      sc.ctypes.data_as(ctypes.c_void_p), off.ctypes.data_as(ctypes.c_void_p),
                                      mul.ctypes.data_as(ctypes.c_void_p), so.ctypes.data_as(ctypes.c_void_p))
    if rc != SG_OK:
        raise RuntimeError(f"sg_compute_normalization failed ({rc})")
    return off, mul, so
