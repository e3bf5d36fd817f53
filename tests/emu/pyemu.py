# TEST INFRASTRUCTURE: host emulation of the kernel's per-packet body.
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_libs = {}


def lib(variant: str = ""):
    """variant "" = the product window; "w32" = a 32-byte header window."""
    if variant not in _libs:
        p = os.environ.get("DPEMU_LIB") if not variant else None
        if not p:
            p = os.path.join(HERE, "build", f"libdpemu{'_' + variant if variant else ''}.so")
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        l = C.CDLL(p)
        V = C.c_void_p
        l.dpemu_process.argtypes = [V, V, C.c_uint64, V, V, C.c_uint32]
        l.dpemu_image_bytes.argtypes = [V]
        l.dpemu_image_bytes.restype = C.c_uint64
        _libs[variant] = l
    return _libs[variant]


def process(tables_ptr, buf: np.ndarray, inp: np.ndarray, out_dtype, variant: str = ""):
    out = np.zeros(len(inp), dtype=out_dtype)
    rc = lib(variant).dpemu_process(C.cast(tables_ptr, C.c_void_p), buf.ctypes.data, buf.nbytes,
                             inp.ctypes.data, out.ctypes.data, len(inp))
    if rc != 0:
        raise RuntimeError(f"emu rejected tables rc={rc}")
    return out


def classifier_forms(variant: str = ""):
    """(bit-vector groups, candidate-list groups) of the last image build on
    this thread (dp_tables.cpp dpd_debug_classifier_forms)."""
    out = (C.c_uint32 * 2)()
    lib(variant).dpd_debug_classifier_forms(out)
    return int(out[0]), int(out[1])
