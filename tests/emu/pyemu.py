# TEST INFRASTRUCTURE: host emulation of the kernel's per-packet body.
import ctypes as C
import os
import subprocess

import numpy as np

from dataplane_amd import _abi as A

HERE = os.path.dirname(os.path.abspath(__file__))
_libs = {}


def lib(variant: str = ""):
    """variant "" = the product window; "w32" = a 32-byte header window;
    "outline" = every device function out of line (DP_EMU_OUTLINE)."""
    if variant not in _libs:
        p = os.environ.get("DPEMU_LIB") if not variant else None
        if not p:
            p = os.path.join(HERE, "build", f"libdpemu{'_' + variant if variant else ''}.so")
            subprocess.run(["make", "-s", "-C", HERE], check=True)
        l = C.CDLL(p)
        V = C.c_void_p
        l.dpemu_process.argtypes = [V, V, C.c_uint64, V, V, V, C.c_uint32]
        l.dpemu_image_bytes.argtypes = [V]
        l.dpemu_image_bytes.restype = C.c_uint64
        _libs[variant] = l
    return _libs[variant]


_libc = C.CDLL(None)
_libc.mprotect.argtypes = [C.c_void_p, C.c_size_t, C.c_int]


def guarded_copy(buf: np.ndarray):
    """A copy of `buf` that ends exactly at a PROT_NONE page (and has one in
    front of its first page): any read or write past the burst buffer faults
    on the host, as it would on the GPU.  Returns (mapping, view)."""
    import mmap
    pg = mmap.PAGESIZE
    npg = max(1, (buf.nbytes + pg - 1) // pg)
    m = mmap.mmap(-1, (npg + 2) * pg)
    base = C.addressof(C.c_char.from_buffer(m))
    if _libc.mprotect(base, pg, 0) or _libc.mprotect(base + (npg + 1) * pg, pg, 0):
        raise OSError("mprotect failed")
    v = np.frombuffer(m, dtype=np.uint8, count=buf.nbytes, offset=(npg + 1) * pg - buf.nbytes)
    v[:] = buf
    return m, v


def process(tables_ptr, buf: np.ndarray, inp: np.ndarray, variant: str = ""):
    """The kernel body over one burst, in place: PKT_RES records.  The body
    runs on a guard-paged copy of the buffer (guarded_copy)."""
    out = np.zeros(len(inp), dtype=A.PKT_OUT)
    meta = np.zeros(len(inp), dtype=A.PKT_META)
    keep, g = guarded_copy(buf)
    rc = lib(variant).dpemu_process(C.cast(tables_ptr, C.c_void_p), g.ctypes.data, buf.nbytes,
                                    inp.ctypes.data, out.ctypes.data, meta.ctypes.data, len(inp))
    buf[:] = g
    del g
    keep.close()
    if rc != 0:
        raise RuntimeError(f"emu rejected tables rc={rc}")
    return A.join_results(out, meta)


def classifier_forms(variant: str = ""):
    """(bit-vector groups, candidate-list groups) of the last image build on
    this thread (dp_tables.cpp dpd_debug_classifier_forms)."""
    out = (C.c_uint32 * 2)()
    lib(variant).dpd_debug_classifier_forms(out)
    return int(out[0]), int(out[1])


def aligned_copy(buf: np.ndarray) -> np.ndarray:
    """16-byte aligned copy of a burst buffer with 16 bytes of slack."""
    raw = np.zeros(buf.nbytes + 48, dtype=np.uint8)
    off = (-raw.ctypes.data) & 15
    a = raw[off:off + buf.nbytes + 16]
    a[:buf.nbytes] = buf
    return a


class ParallelEmu:
    """The kernel body over one compiled image on host threads (bench.py's
    compiled CPU leg); libdpemu_fast.so is the -O3 build."""

    def __init__(self, tables_ptr):
        p = os.path.join(HERE, "build", "libdpemu_fast.so")
        if not os.path.exists(p):
            subprocess.run(["make", "-s", "-C", HERE, "build/libdpemu_fast.so"], check=True)
        self.l = l = C.CDLL(p)
        V = C.c_void_p
        l.dpemu_ctx_create.argtypes = [V]
        l.dpemu_ctx_create.restype = V
        l.dpemu_ctx_free.argtypes = [V]
        l.dpemu_run_parallel.argtypes = [V, V, C.c_uint64, V, V, V, C.c_uint32, C.c_uint32,
                                         C.c_uint32]
        self.h = l.dpemu_ctx_create(C.cast(tables_ptr, C.c_void_p))
        if not self.h:
            raise RuntimeError("emu rejected tables")

    def run(self, buf: np.ndarray, buf_bytes: int, inp: np.ndarray, out: np.ndarray, threads: int,
            burst: int = 64, meta: np.ndarray = None):
        """`out` a PKT_OUT array, `meta` an optional PKT_META one."""
        rc = self.l.dpemu_run_parallel(self.h, buf.ctypes.data, buf_bytes, inp.ctypes.data,
                                       out.ctypes.data,
                                       meta.ctypes.data if meta is not None else None,
                                       len(inp), burst, threads)
        if rc != 0:
            raise RuntimeError(f"emu run rc={rc}")

    def close(self):
        if self.h:
            self.l.dpemu_ctx_free(self.h)
            self.h = None
