"""A stand-in for an rte_mempool of rte_mbufs (test infrastructure).

Each element is laid out like a DPDK pktmbuf pool element: a 128-byte
rte_mbuf header (the DP_MBUF_LAYOUT_DPDK fields written at their
rte_mbuf_core.h offsets), then the data buffer: RTE_PKTMBUF_HEADROOM (128 B)
and a 2048-byte data room.  The region is any numpy uint8 array -- ordinary
memory for the host-only tests, pinned memory for the GPU tests.
"""
from __future__ import annotations

import struct

import numpy as np

HDR = 128
HEADROOM = 128
ROOM = 2048
STRIDE = HDR + HEADROOM + ROOM


class FakeMempool:
    def __init__(self, mem: np.ndarray):
        self.mem = mem
        self.base = mem.ctypes.data
        self.n = mem.nbytes // STRIDE

    @staticmethod
    def bytes_for(n: int) -> int:
        return n * STRIDE

    def addr(self, i: int) -> int:
        return self.base + i * STRIDE

    def _put(self, i: int, off: int, fmt: str, v) -> None:
        o = i * STRIDE + off
        self.mem[o:o + struct.calcsize(fmt)] = np.frombuffer(struct.pack(fmt, v), np.uint8)

    def _get(self, i: int, off: int, fmt: str):
        o = i * STRIDE + off
        return struct.unpack(fmt, self.mem[o:o + struct.calcsize(fmt)].tobytes())[0]

    def load(self, frames, ports) -> np.ndarray:
        """rte_pktmbuf_alloc + copy of each frame (as a NIC rx would leave it);
        returns the mbuf addresses of the burst."""
        assert len(frames) <= self.n
        for i, (f, p) in enumerate(zip(frames, ports)):
            buf = self.addr(i) + HDR
            self._put(i, 0, "<Q", buf)                 # buf_addr
            self._put(i, 8, "<Q", 0)                   # buf_iova
            self._put(i, 16, "<H", HEADROOM)           # data_off
            self._put(i, 18, "<H", 1)                  # refcnt
            self._put(i, 20, "<H", 1)                  # nb_segs
            self._put(i, 22, "<H", int(p))             # port
            self._put(i, 36, "<I", len(f))             # pkt_len
            self._put(i, 40, "<H", len(f))             # data_len
            self._put(i, 54, "<H", HEADROOM + ROOM)    # buf_len
            o = i * STRIDE + HDR + HEADROOM
            self.mem[o:o + len(f)] = np.frombuffer(f, np.uint8)
        return np.array([self.addr(i) for i in range(len(frames))], dtype=np.uint64)

    def field(self, i: int, name: str) -> int:
        off, fmt = {"data_off": (16, "<H"), "data_len": (40, "<H"), "pkt_len": (36, "<I"),
                    "port": (22, "<H"), "nb_segs": (20, "<H")}[name]
        return self._get(i, off, fmt)

    def set_field(self, i: int, name: str, v: int) -> None:
        off, fmt = {"data_off": (16, "<H"), "data_len": (40, "<H"), "pkt_len": (36, "<I"),
                    "port": (22, "<H"), "nb_segs": (20, "<H"), "buf_addr": (0, "<Q")}[name]
        self._put(i, off, fmt, v)

    def frame(self, i: int) -> bytes:
        """Mbuf::raw_data (dpdk/src/mem.rs:502-522)."""
        o = i * STRIDE + HDR + self.field(i, "data_off")
        return self.mem[o:o + self.field(i, "data_len")].tobytes()
