# SPDX-License-Identifier: Apache-2.0
"""Seeded synthetic workloads via the native generator.

A `Workload` owns lowered tables (a `dp_tables_desc_t` pointer valid while
the workload lives) and a burst: a 16-byte aligned frame buffer with
DP_HEADROOM bytes in front of every frame plus the `dp_pkt_in_t` records.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi as A

# B_pkt of SURVEY.md §8d: L_in + L_out + 8 (in-meta) + 8 (out-meta)
ALGO_BYTES = {1: 136.0, 2: 136.0, 3: 715.7, 4: 236.0, 5: 144.0}

CONFIG_NAMES = {
    1: "64B IPv4/UDP synthetic burst, 1k-route LPM only",
    2: "64B IPv4/UDP, 1M-route LPM + 10k-rule ACL + NAT",
    3: "IMIX (64/570/1518B) IPv4, 1M-route LPM + 10k ACL + NAT",
    4: "VXLAN-encapped IPv4 inner: decap + LPM + NAT + re-encap",
    5: "IPv4+IPv6 mix, 1M v4 + 200k v6 routes, 10k ACL, NAT",
}


class Workload:
    def __init__(self, config: int, n_packets: int, seed: int = 1, n_routes_v4: int = 0,
                 n_routes_v6: int = 0, n_acl: int = 0, n_nat: int = 0, n_vni: int = 0,
                 tcp_percent: int = 0, layout: str = "packed"):
        """layout "packed": DP_HEADROOM (96 B, the reference test buffer) in
        front of 16-byte aligned frames; "dpdk": DPDK mbuf data layout,
        RTE_PKTMBUF_HEADROOM (128 B) in front of 64-byte aligned frames."""
        self._lib = A.work_lib()
        cfg = A.WorkloadConfig(config=config, n_packets=n_packets, seed=seed,
                               n_routes_v4=n_routes_v4, n_routes_v6=n_routes_v6, n_acl=n_acl,
                               n_nat=n_nat, n_vni=n_vni, tcp_percent=tcp_percent,
                               layout={"packed": 0, "dpdk": 1}[layout])
        h = C.c_void_p()
        A.check(self._lib.dpw_build(C.byref(cfg), C.byref(h)), "dpw_build")
        self._h = h
        self.config = config
        self.n = int(self._lib.dpw_n(h))
        nbytes = int(self._lib.dpw_buf_bytes(h))
        self.tables = self._lib.dpw_tables(h)  # POINTER(TablesDesc)
        raw = np.ctypeslib.as_array(self._lib.dpw_buf(h), shape=(nbytes,))
        self.buf = raw.copy()
        inp = C.cast(self._lib.dpw_in(h), C.POINTER(C.c_uint8))
        self.inp = np.ctypeslib.as_array(inp, shape=(self.n * 16,)).view(A.PKT_IN).copy()
        self.frame_bytes = int(self._lib.dpw_frame_bytes(h))

    def fresh_buf(self) -> np.ndarray:
        return self.buf.copy()

    def close(self):
        if self._h:
            self._lib.dpw_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
