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

from dataplane_amd import _abi as A

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
        l.dpo_tables_build2.argtypes = [V, V, C.POINTER(V)]
        l.dpo_portfw_rule_alive.argtypes = [V, C.c_uint32]
        l.dpo_flows_set_clock.argtypes = [V, C.c_uint64]
        l.dpo_flows_sync.argtypes = [V, V]
        l.dpo_tables_free.argtypes = [V]
        l.dpo_process_burst.argtypes = [V, V, C.c_uint64, V, V, V, C.c_uint32, V]
        l.dpo_process_parallel.argtypes = [V, V, C.c_uint64, V, V, V, C.c_uint32, C.c_uint32,
                                           C.c_uint32]
        l.dpo_lpm.argtypes = [V, C.c_uint32, C.c_uint8, V]
        l.dpo_lpm.restype = C.c_int64
        l.dpo_acl_lookup.argtypes = [V, C.c_uint8, C.c_uint8, C.c_uint32, C.c_uint32, V, V,
                                     C.c_int, C.c_uint16, C.c_uint16]
        l.dpo_acl_lookup.restype = C.c_int64
        l.dpo_acl_classify.argtypes = [V, V, V, C.c_uint32]
        l.dpo_ff_classify.argtypes = [V, V, V, C.c_uint32, C.c_int]
        l.dpo_nat_lookup.argtypes = [V, C.c_uint32, C.c_uint32, C.c_uint32, V, C.c_int,
                                     C.c_uint16, V, V]
        l.dpo_checksum_ipv4_header.argtypes = [V, C.c_uint32]
        l.dpo_checksum_ipv4_header.restype = C.c_uint16
        l.dpo_hash_bytes.argtypes = [V, C.c_uint32]
        l.dpo_hash_bytes.restype = C.c_uint64
        l.dpo_reserialize.argtypes = [V, C.c_uint32, V, C.c_uint32]
        l.dpo_reserialize.restype = C.c_int
        l.dpo_process_burst_flows.argtypes = [V, V, V, C.c_uint64, V, V, V, C.c_uint32, V]
        l.dpo_flows_create.argtypes = [C.POINTER(V)]
        l.dpo_flows_free.argtypes = [V]
        l.dpo_flows_set_capacity.argtypes = [V, C.c_uint64]
        l.dpo_flow_insert.argtypes = [V, V, C.c_uint32, V, V]
        l.dpo_flow_insert_pair.argtypes = [V, V, V, V, V]
        l.dpo_flow_lookup.argtypes = [V, V, C.c_uint32, V]
        l.dpo_flow_get.argtypes = [V, V, C.c_uint32, V]
        l.dpo_flow_remove.argtypes = [V, V, C.c_uint32, V]
        l.dpo_flow_invalidate.argtypes = [V, V, C.c_uint32]
        l.dpo_flow_set_status.argtypes = [V, C.c_uint64, C.c_uint32]
        l.dpo_flow_sweep.argtypes = [V, C.c_uint64, V]
        l.dpo_flow_count.argtypes = [V, V, V]
        _lib = l
    return _lib


class Oracle:
    def __init__(self, tables_ptr, prev: "Oracle | None" = None):
        """`prev`: the previous generation on the same device (port-forwarding
        entries carry over as PortFwTable::update keeps them)."""
        h = C.c_void_p()
        rc = lib().dpo_tables_build2(C.cast(tables_ptr, C.c_void_p), prev.h if prev else None,
                                     C.byref(h))
        if rc != 0:
            raise ValueError(f"oracle rejected tables: rc={rc}")
        self.h = h

    def rule_alive(self, rule_id: int) -> bool:
        """Does port-forwarding entry `rule_id` live in these tables?"""
        return bool(lib().dpo_portfw_rule_alive(self.h, rule_id))

    def acl_classify(self, keys: np.ndarray) -> np.ndarray:
        """AclFilter's decision per A.ACL_KEY record (dpgpu.h dp_acl_classify)."""
        keys = np.ascontiguousarray(keys, dtype=A.ACL_KEY)
        out = np.zeros(len(keys), dtype=A.ACL_RESULT)
        if lib().dpo_acl_classify(self.h, keys.ctypes.data, out.ctypes.data, len(keys)) != 0:
            raise RuntimeError("oracle acl_classify failed")
        return out

    def ff_classify(self, inputs: np.ndarray, stage: int = 0) -> np.ndarray:
        """FlowFilterContext::lookup_batch per A.FF_INPUT record (dpgpu.h
        dp_ff_classify); stage 1 / 2: the remote / local rules alone."""
        inputs = np.ascontiguousarray(np.atleast_1d(inputs), dtype=A.FF_INPUT)
        out = np.zeros(len(inputs), dtype=A.FF_RESULT)
        if lib().dpo_ff_classify(self.h, inputs.ctypes.data, out.ctypes.data, len(inputs), stage) != 0:
            raise RuntimeError("oracle ff_classify failed")
        return out

    def process(self, buf: np.ndarray, inp: np.ndarray, stats: bool = False):
        """One burst, in place: PKT_RES records (dp_pkt_out_t + dp_pkt_meta_t)."""
        out = np.zeros(len(inp), dtype=A.PKT_OUT)
        meta = np.zeros(len(inp), dtype=A.PKT_META)
        st = np.zeros(34, dtype=np.uint64)
        rc = lib().dpo_process_burst(self.h, buf.ctypes.data, buf.nbytes, inp.ctypes.data,
                                     out.ctypes.data, meta.ctypes.data, len(inp), st.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"oracle process failed rc={rc}")
        res = A.join_results(out, meta)
        return (res, st) if stats else res

    def process_flows(self, buf: np.ndarray, inp: np.ndarray, flows, stats=False):
        """One burst with FlowLookup on `flows` (an OracleFlows, or None for an
        empty flow table): (PKT_RES records, flow_refs[, stats]); flow_refs is
        the records' flow_ref column (PacketMeta.flow_info)."""
        out = np.zeros(len(inp), dtype=A.PKT_OUT)
        meta = np.zeros(len(inp), dtype=A.PKT_META)
        st = np.zeros(34, dtype=np.uint64)
        rc = lib().dpo_process_burst_flows(self.h, flows.h if flows is not None else None,
                                           buf.ctypes.data, buf.nbytes, inp.ctypes.data,
                                           out.ctypes.data, meta.ctypes.data, len(inp),
                                           st.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"oracle process failed rc={rc}")
        res = A.join_results(out, meta)
        refs = res["flow_ref"].copy()
        return (res, refs, st) if stats else (res, refs)

    def process_parallel(self, buf, inp, out, threads: int, burst: int = 64, meta=None):
        """CPU baseline: `out` a PKT_OUT array, `meta` an optional PKT_META one."""
        rc = lib().dpo_process_parallel(self.h, buf.ctypes.data, buf.nbytes, inp.ctypes.data,
                                        out.ctypes.data,
                                        meta.ctypes.data if meta is not None else None,
                                        len(inp), burst, threads)
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


class OracleFlows:
    """The oracle's FlowTable with the interface of dataplane_amd.flows.FlowTable."""

    def __init__(self):
        h = C.c_void_p()
        lib().dpo_flows_create(C.byref(h))
        self.h = h

    def _chk(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"oracle {what} rc={rc}")

    def set_capacity(self, capacity: int) -> None:
        self._chk(lib().dpo_flows_set_capacity(self.h, capacity), "set_capacity")

    def set_clock(self, now_ns: int) -> None:
        """Instant::now() for the bursts that follow (DP_OPT_CLOCK)."""
        self._chk(lib().dpo_flows_set_clock(self.h, now_ns), "set_clock")

    def sync(self, oracle: "Oracle") -> None:
        """update_nat_allocator for `oracle`'s tables (what dp_tables_publish does
        for the flow tables attached on the device)."""
        self._chk(lib().dpo_flows_sync(self.h, oracle.h), "sync")

    def insert(self, flows):
        from dataplane_amd import _abi as A
        flows = np.ascontiguousarray(np.atleast_1d(flows), dtype=A.FLOW)
        refs = np.zeros(len(flows), np.uint64)
        res = np.zeros(len(flows), np.int32)
        self._chk(lib().dpo_flow_insert(self.h, flows.ctypes.data, len(flows), refs.ctypes.data,
                                        res.ctypes.data), "insert")
        return refs, res

    def insert_pair(self, a, b):
        from dataplane_amd import _abi as A
        a = np.ascontiguousarray(a, dtype=A.FLOW)
        b = np.ascontiguousarray(b, dtype=A.FLOW)
        refs = np.zeros(2, np.uint64)
        res = np.zeros(2, np.int32)
        self._chk(lib().dpo_flow_insert_pair(self.h, a.ctypes.data, b.ctypes.data,
                                             refs.ctypes.data, res.ctypes.data), "insert_pair")
        return refs, res

    def lookup(self, keys):
        from dataplane_amd import _abi as A
        keys = np.ascontiguousarray(np.atleast_1d(keys), dtype=A.FLOW_KEY)
        out = np.zeros(len(keys), A.FLOW_INFO)
        self._chk(lib().dpo_flow_lookup(self.h, keys.ctypes.data, len(keys), out.ctypes.data),
                  "lookup")
        return out

    def get(self, refs):
        from dataplane_amd import _abi as A
        refs = np.ascontiguousarray(refs, dtype=np.uint64)
        out = np.zeros(len(refs), A.FLOW_INFO)
        self._chk(lib().dpo_flow_get(self.h, refs.ctypes.data, len(refs), out.ctypes.data), "get")
        return out

    def remove(self, keys) -> int:
        from dataplane_amd import _abi as A
        keys = np.ascontiguousarray(np.atleast_1d(keys), dtype=A.FLOW_KEY)
        n = C.c_uint32()
        self._chk(lib().dpo_flow_remove(self.h, keys.ctypes.data, len(keys), C.byref(n)), "remove")
        return n.value

    def invalidate(self, refs) -> None:
        refs = np.ascontiguousarray(refs, dtype=np.uint64)
        self._chk(lib().dpo_flow_invalidate(self.h, refs.ctypes.data, len(refs)), "invalidate")

    def set_status(self, ref: int, status: int) -> None:
        self._chk(lib().dpo_flow_set_status(self.h, int(ref), status), "set_status")

    def sweep(self, now: int) -> int:
        n = C.c_uint64()
        self._chk(lib().dpo_flow_sweep(self.h, now, C.byref(n)), "sweep")
        return n.value

    def count(self):
        ln, act = C.c_uint64(), C.c_uint64()
        self._chk(lib().dpo_flow_count(self.h, C.byref(ln), C.byref(act)), "count")
        return ln.value, act.value

    def close(self):
        if self.h:
            lib().dpo_flows_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
