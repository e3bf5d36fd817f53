# TEST INFRASTRUCTURE: host emulation of the kernel's per-packet body.
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        p = os.path.join(HERE, "build", "libdpemu.so")
        subprocess.run(["make", "-s", "-C", HERE], check=True)
        l = C.CDLL(p)
        V = C.c_void_p
        l.dpemu_process.argtypes = [V, V, C.c_uint64, V, V, C.c_uint32]
        l.dpemu_image_bytes.argtypes = [V]
        l.dpemu_image_bytes.restype = C.c_uint64
        _lib = l
    return _lib


def process(tables_ptr, buf: np.ndarray, inp: np.ndarray, out_dtype):
    out = np.zeros(len(inp), dtype=out_dtype)
    rc = lib().dpemu_process(C.cast(tables_ptr, C.c_void_p), buf.ctypes.data, buf.nbytes,
                             inp.ctypes.data, out.ctypes.data, len(inp))
    if rc != 0:
        raise RuntimeError(f"emu rejected tables rc={rc}")
    return out
