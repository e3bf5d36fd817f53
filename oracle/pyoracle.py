# SPDX-License-Identifier: Apache-2.0
"""TEST INFRASTRUCTURE -- NOT PRODUCT CODE.

ctypes binding of oracle/build/libdporacle.so, the C++ restatement of the
reference pipeline (see oracle/dp_oracle.h for what pins it).  Imported only
by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        p = os.path.join(HERE, "build", "libdporacle.so")
        if not os.path.exists(p):
            raise RuntimeError("oracle not built: make -C oracle")
        l = C.CDLL(p)
        V = C.c_void_p
        l.dpo_tables_build.argtypes = [V, C.POINTER(V)]
        l.dpo_tables_free.argtypes = [V]
        l.dpo_process_burst.argtypes = [V, V, C.c_uint64, V, V, C.c_uint32, V]
        l.dpo_process_parallel.argtypes = [V, V, C.c_uint64, V, V, C.c_uint32, C.c_uint32,
                                           C.c_uint32]
        l.dpo_lpm.argtypes = [V, C.c_uint32, C.c_uint8, V]
        l.dpo_lpm.restype = C.c_int64
        l.dpo_acl_lookup.argtypes = [V, C.c_uint8, C.c_uint8, C.c_uint32, C.c_uint32, V, V,
                                     C.c_int, C.c_uint16, C.c_uint16]
        l.dpo_acl_lookup.restype = C.c_int64
        l.dpo_nat_lookup.argtypes = [V, C.c_uint32, C.c_uint32, C.c_uint32, V, C.c_int,
                                     C.c_uint16, V, V]
        l.dpo_checksum_ipv4_header.argtypes = [V, C.c_uint32]
        l.dpo_checksum_ipv4_header.restype = C.c_uint16
        l.dpo_hash_bytes.argtypes = [V, C.c_uint32]
        l.dpo_hash_bytes.restype = C.c_uint64
        l.dpo_reserialize.argtypes = [V, C.c_uint32, V, C.c_uint32]
        l.dpo_reserialize.restype = C.c_int
        _lib = l
    return _lib


class Oracle:
    def __init__(self, tables_ptr):
        h = C.c_void_p()
        rc = lib().dpo_tables_build(C.cast(tables_ptr, C.c_void_p), C.byref(h))
        if rc != 0:
            raise ValueError(f"oracle rejected tables: rc={rc}")
        self.h = h

    def process(self, buf: np.ndarray, inp: np.ndarray, out_dtype, stats: bool = False):
        out = np.zeros(len(inp), dtype=out_dtype)
        st = np.zeros(34, dtype=np.uint64)
        rc = lib().dpo_process_burst(self.h, buf.ctypes.data, buf.nbytes, inp.ctypes.data,
                                     out.ctypes.data, len(inp), st.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"oracle process failed rc={rc}")
        return (out, st) if stats else out

    def process_parallel(self, buf, inp, out, threads: int, burst: int = 64):
        rc = lib().dpo_process_parallel(self.h, buf.ctypes.data, buf.nbytes, inp.ctypes.data,
                                        out.ctypes.data, len(inp), burst, threads)
        if rc != 0:
            raise RuntimeError(f"oracle parallel failed rc={rc}")

    def close(self):
        if self.h:
            lib().dpo_tables_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def reserialize(frame: bytes) -> bytes | None:
    """Packet::new + Packet::serialize of one frame (None: does not parse)."""
    out = (C.c_uint8 * (len(frame) + 256))()
    n = lib().dpo_reserialize(frame, len(frame), out, len(out))
    return None if n < 0 else bytes(out[:n])
