# SPDX-License-Identifier: Apache-2.0
"""Host mirror of the flow table API (include/dpgpu.h "Flow table").

``FlowTable`` replaces the reference's ``Arc<FlowTable>``
(flow-entry/src/flow_table/table.rs:24-330): the table lives in HBM on one
device and is shared by every context it is attached to (``GpuPathNf.attach_flows``,
the analogue of ``FlowLookup::new(name, flow_table)``,
flow-entry/src/flow_table/nf_lookup.rs:24-32).  Keys and flows are numpy
records of ``_abi.FLOW_KEY`` / ``_abi.FLOW`` so batches go to the library as
one array.
"""
from __future__ import annotations

import ctypes as C
import ipaddress
from typing import Optional, Sequence

import numpy as np

from . import _abi as A

NEVER = (1 << 63) - 1  # expires_at of a flow whose timer never fires in a test


def _addr(a) -> tuple:
    ip = ipaddress.ip_address(a)
    b = ip.packed
    return ip.version, b + bytes(16 - len(b))


def flow_key(src_vni: int, src, dst, kind: int, sport: int = 0, dport: int = 0) -> np.ndarray:
    """FlowKey::new(src_vpcd, src_ip, dst_ip, proto_key_info)
    (net/src/flows/flow_key.rs:465-483); ``src_vni`` 0 = no source VPC."""
    fs, sb = _addr(src)
    fd, db = _addr(dst)
    if fs != fd:
        raise ValueError("flow key addresses of different families")
    k = np.zeros((), dtype=A.FLOW_KEY)
    k["src_vni"], k["family"], k["kind"] = src_vni, 4 if fs == 4 else 6, kind
    k["sport"], k["dport"] = sport, dport
    k["src"] = np.frombuffer(sb, np.uint8)
    k["dst"] = np.frombuffer(db, np.uint8)
    return k


def reverse_key(k: np.ndarray, src_vni: int) -> np.ndarray:
    """FlowKey::reverse(src_vpcd) (flow_key.rs:567-576)."""
    r = k.copy()
    r["src_vni"] = src_vni
    r["src"], r["dst"] = k["dst"], k["src"]
    if int(k["kind"]) in (A.FLOW_TCP, A.FLOW_UDP):
        r["sport"], r["dport"] = k["dport"], k["sport"]
    return r


def make_flow(key: np.ndarray, dst_vni: int, flags: int = 0, genid: int = 0,
              expires_at: int = NEVER) -> np.ndarray:
    f = np.zeros((), dtype=A.FLOW)
    f["key"], f["dst_vni"], f["flags"] = key, dst_vni, flags
    f["genid"], f["expires_at"] = genid, expires_at
    return f


class FlowTable:
    """A device flow table (dp_flow_table_create)."""

    def __init__(self, device: int = 0, slots: int = 1 << 16):
        self.lib = A.gpu_lib()
        h = C.c_void_p()
        A.check(self.lib.dp_flow_table_create(device, slots, C.byref(h)), "dp_flow_table_create",
                self.lib)
        self.h = h

    def set_capacity(self, capacity: int) -> None:
        A.check(self.lib.dp_flow_table_set_capacity(self.h, capacity), "set_capacity", self.lib)

    def insert(self, flows: np.ndarray):
        flows = np.ascontiguousarray(np.atleast_1d(flows), dtype=A.FLOW)
        refs = np.zeros(len(flows), np.uint64)
        res = np.zeros(len(flows), np.int32)
        A.check(self.lib.dp_flow_insert(self.h, flows.ctypes.data, len(flows), refs.ctypes.data,
                                        res.ctypes.data), "dp_flow_insert", self.lib)
        return refs, res

    def insert_pair(self, a: np.ndarray, b: np.ndarray):
        a = np.ascontiguousarray(a, dtype=A.FLOW)
        b = np.ascontiguousarray(b, dtype=A.FLOW)
        refs = np.zeros(2, np.uint64)
        res = np.zeros(2, np.int32)
        A.check(self.lib.dp_flow_insert_pair(self.h, a.ctypes.data, b.ctypes.data,
                                             refs.ctypes.data, res.ctypes.data),
                "dp_flow_insert_pair", self.lib)
        return refs, res

    def lookup(self, keys: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(np.atleast_1d(keys), dtype=A.FLOW_KEY)
        out = np.zeros(len(keys), A.FLOW_INFO)
        A.check(self.lib.dp_flow_lookup(self.h, keys.ctypes.data, len(keys), out.ctypes.data),
                "dp_flow_lookup", self.lib)
        return out

    def get(self, refs: Sequence[int]) -> np.ndarray:
        refs = np.ascontiguousarray(refs, dtype=np.uint64)
        out = np.zeros(len(refs), A.FLOW_INFO)
        A.check(self.lib.dp_flow_get(self.h, refs.ctypes.data, len(refs), out.ctypes.data),
                "dp_flow_get", self.lib)
        return out

    def remove(self, keys: np.ndarray) -> int:
        keys = np.ascontiguousarray(np.atleast_1d(keys), dtype=A.FLOW_KEY)
        n = C.c_uint32()
        A.check(self.lib.dp_flow_remove(self.h, keys.ctypes.data, len(keys), C.byref(n)),
                "dp_flow_remove", self.lib)
        return n.value

    def invalidate(self, refs: Sequence[int]) -> None:
        refs = np.ascontiguousarray(refs, dtype=np.uint64)
        A.check(self.lib.dp_flow_invalidate(self.h, refs.ctypes.data, len(refs)),
                "dp_flow_invalidate", self.lib)

    def set_status(self, ref: int, status: int) -> None:
        A.check(self.lib.dp_flow_set_status(self.h, int(ref), status), "dp_flow_set_status",
                self.lib)

    def sweep(self, now: int) -> int:
        n = C.c_uint64()
        A.check(self.lib.dp_flow_sweep(self.h, now, C.byref(n)), "dp_flow_sweep", self.lib)
        return n.value

    def count(self) -> tuple:
        ln, act = C.c_uint64(), C.c_uint64()
        A.check(self.lib.dp_flow_count(self.h, C.byref(ln), C.byref(act)), "dp_flow_count",
                self.lib)
        return ln.value, act.value

    def debug_stats(self) -> dict:
        """Slot census (test hook dpf_debug_table_stats, not part of dpgpu.h):
        FULL / TOMB / EMPTY slots and the lookup probe bound."""
        out = (C.c_uint64 * 4)()
        self.lib.dpf_debug_table_stats.argtypes = [C.c_void_p, C.c_void_p]
        A.check(self.lib.dpf_debug_table_stats(self.h, out), "dpf_debug_table_stats", self.lib)
        return dict(full=out[0], tomb=out[1], empty=out[2], max_probe=out[3])

    def close(self) -> None:
        if self.h:
            self.lib.dp_flow_table_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def burst_request_flows(buf: np.ndarray, inp: np.ndarray, sel: np.ndarray, dst_vni: np.ndarray,
                        genid: int, flags: int = A.FLOW_INITIATOR) -> np.ndarray:
    """Flows (one per distinct key) for the packets `sel` of a burst of
    untagged Eth / IPv4 (no options) / TCP|UDP frames seeded with their
    source VNI: FlowKey::try_from of each packet, its destination VPC
    `dst_vni[i]`, `genid`, never expiring.  Vectorised; other frames are
    skipped."""
    off = inp["off"].astype(np.int64)
    sel = np.asarray(sel)
    o = off[sel]
    proto = buf[o + 23]
    keep = (buf[o + 12] == 8) & (buf[o + 13] == 0) & (buf[o + 14] == 0x45) & \
           ((proto == 6) | (proto == 17)) & (inp["src_vni"][sel] != 0) & (dst_vni[sel] != 0)
    sel, o, proto = sel[keep], o[keep], proto[keep]
    fl = np.zeros(len(sel), A.FLOW)
    k = fl["key"]
    k["src_vni"] = inp["src_vni"][sel]
    k["family"] = 4
    k["kind"] = np.where(proto == 6, A.FLOW_TCP, A.FLOW_UDP)
    k["sport"] = (buf[o + 34].astype(np.uint16) << 8) | buf[o + 35]
    k["dport"] = (buf[o + 36].astype(np.uint16) << 8) | buf[o + 37]
    for j in range(4):
        k["src"][:, j] = buf[o + 26 + j]
        k["dst"][:, j] = buf[o + 30 + j]
    fl["dst_vni"] = dst_vni[sel]
    fl["flags"] = flags
    fl["genid"] = genid
    fl["expires_at"] = NEVER
    kb = np.ascontiguousarray(fl["key"]).view(np.uint8).reshape(len(fl), -1)
    _, first = np.unique(kb, axis=0, return_index=True)
    return fl[np.sort(first)]


def key_records(keys: Sequence[np.ndarray]) -> np.ndarray:
    out = np.zeros(len(keys), A.FLOW_KEY)
    for i, k in enumerate(keys):
        out[i] = k
    return out


def none_if_absent(ref: int) -> Optional[int]:
    return None if int(ref) == A.FLOW_NONE else int(ref)
