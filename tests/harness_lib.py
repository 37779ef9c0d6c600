"""ctypes binding of harness/build/libsiril_harness.so: the reference-side glue
(harness/siril_glue.c: stack_* and register_shift_dft with the reference's signatures) plus the
GTK-free environment it runs in (harness/siril_env.c)."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "harness", "build", "libsiril_harness.so")
CLI = os.path.join(ROOT, "harness", "build", "siril_cli")
P = ctypes.c_void_p
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "harness")], check=True)
    lib = ctypes.CDLL(LIB)
    lib.harness_open_ser.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.harness_open_ser.restype = P
    lib.harness_open_fits.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.c_int]
    lib.harness_open_fits.restype = P
    lib.harness_close.argtypes = [P]
    lib.harness_stack.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_int, ctypes.c_int]
    lib.harness_register.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.harness_get_regdata.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
    lib.harness_set_regdata.argtypes = [P, ctypes.c_int, P, P]
    lib.harness_set_registration_layer.argtypes = [ctypes.c_int]
    lib.harness_set_max_thread.argtypes = [ctypes.c_int]
    lib.harness_set_cancel_after.argtypes = [ctypes.c_int]
    lib.harness_set_fail_read.argtypes = [ctypes.c_int]
    lib.harness_set_reference_image.argtypes = [P, ctypes.c_int]
    lib.harness_set_included.argtypes = [P, ctypes.c_int, ctypes.c_int]
    lib.harness_gfit_shape.argtypes = [ctypes.POINTER(ctypes.c_int)] * 3
    lib.harness_gfit_copy.argtypes = [P, ctypes.c_size_t]
    lib.harness_gfit_hi.restype = ctypes.c_ushort
    lib.harness_save_gfit.argtypes = [ctypes.c_char_p]
    lib.siril_gpu_release.restype = None
    lib.harness_set_run_in_thread.argtypes = [ctypes.c_int]
    lib.harness_gfit_exposure.restype = ctypes.c_double
    lib.harness_set_devices.argtypes = [ctypes.c_int, P]
    _lib = lib
    return lib


class Sequence:
    """a sequence struct (harness/siril_compat.h) opened through siril_env.c"""

    def __init__(self, handle, shape):
        self.h = handle
        self.shape = shape

    @classmethod
    def ser(cls, path, debayer=-2, shape=None):
        h = load().harness_open_ser(os.fsencode(path), debayer)
        if not h:
            raise OSError(path)
        return cls(h, shape)

    @classmethod
    def fits(cls, paths, shape=None):
        arr = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
        h = load().harness_open_fits(arr, len(paths))
        if not h:
            raise OSError(paths[0])
        return cls(h, shape)

    def close(self):
        if self.h:
            load().harness_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_regdata(self, layer, sx, sy):
        sx = np.ascontiguousarray(sx, np.int32)
        sy = np.ascontiguousarray(sy, np.int32)
        assert load().harness_set_regdata(self.h, layer, sx.ctypes.data_as(P), sy.ctypes.data_as(P)) == 0

    def regdata(self, layer, n):
        lib = load()
        sx, sy, q = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n)
        for i in range(n):
            a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
            if lib.harness_get_regdata(self.h, layer, i, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)):
                return None
            sx[i], sy[i], q[i] = a.value, b.value, c.value
        return sx, sy, q


def set_devices(devs):
    """the glue's context on these device ids (None: every visible device)"""
    lib = load()
    if devs is None:
        return lib.harness_set_devices(-1, None)
    arr = (ctypes.c_int * len(devs))(*devs)
    return lib.harness_set_devices(len(devs), ctypes.cast(arr, P))


def gfit():
    """(C, H, W) planes of the result image the glue handed to gfit"""
    lib = load()
    w, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    assert lib.harness_gfit_shape(ctypes.byref(w), ctypes.byref(h), ctypes.byref(c)) == 0
    out = np.zeros((c.value, h.value, w.value), np.uint16)
    assert lib.harness_gfit_copy(out.ctypes.data_as(P), out.size) == 0
    return out
