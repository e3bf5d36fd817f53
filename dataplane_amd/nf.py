# SPDX-License-Identifier: Apache-2.0
"""Host-side mirror of the reference's stage API for this path.

The reference drives the path through ``NetworkFunction`` stages
(``pipeline/src/static_nf.rs:12-32``)::

    fn process(&mut self, input: impl Iterator<Item = Packet<Buf>>) -> impl Iterator<Item = Packet<Buf>>
    fn set_data(&mut self, data: Arc<PipelineData>)

``GpuPathNf`` keeps that shape: ``process`` materialises the burst (as
``FlowFilter::process`` does, ``flow-filter/src/lib.rs:357-362``), runs the
whole Ingress..Egress + serialize block on the GPU through the C ABI, applies
the returned DoneReason / metadata to every packet and yields them all
(``KEEP`` semantics: packets are marked, never removed).  ``set_data`` carries
the generation id.  Device-resident bursts go through ``process_device``.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Iterable, Iterator, List, Optional

import numpy as np

from . import _abi as A


@dataclass
class PipelineData:
    """pipeline/src/pipeline.rs:22-42"""
    genid: int = 0


@dataclass
class Packet:
    """A frame plus the PacketMeta fields this path reads and writes."""
    frame: bytes
    iif: int = 1
    src_vni: int = 0            # seeded src_vpcd (harness idiom, DP_IN_SEEDED_OVERLAY)
    seeded_overlay: bool = False
    # results (net/src/packet/meta.rs:138-154)
    done: Optional[str] = None
    meta_flags: int = 0
    oif: Optional[int] = None
    dst_vni: Optional[int] = None
    fib_entry: Optional[int] = None
    acl_rule: Optional[int] = None
    vrf: Optional[int] = None           # PacketMeta.vrf
    nh_addr: Optional[str] = None       # PacketMeta.nh_addr (next-hop IP, text form)
    dscp: Optional[int] = None          # PacketMeta.dscp / .ecn (set by the path when known)
    ecn: Optional[int] = None
    flow_ref: int = 0                   # the packet's attached flow (meta.flow_info), 0 = none

    def is_done(self) -> bool:
        return self.done is not None


class GpuPathNf:
    """One context per worker thread (worker.rs:175); one HIP stream each."""

    def __init__(self, device: int = 0, name: str = "gpu-path"):
        self.name = name
        self.lib = A.gpu_lib()
        h = C.c_void_p()
        A.check(self.lib.dp_ctx_create(device, C.byref(h)), "dp_ctx_create", self.lib)
        self.ctx = h
        self.data = PipelineData()
        self._keep = None

    # -- table publication --------------------------------
    def publish(self, tables_ptr) -> None:
        """Publish lowered tables (a POINTER(TablesDesc)); bursts that start
        after this returns see the new generation."""
        A.check(self.lib.dp_tables_publish(self.ctx, tables_ptr), "dp_tables_publish", self.lib)
        self.data.genid = int(self.lib.dp_tables_genid(self.ctx))

    def set_data(self, data: PipelineData) -> None:
        self.data = data

    # -- NetworkFunction::process -------------------------------------------
    def process(self, packets: Iterable[Packet]) -> Iterator[Packet]:
        burst: List[Packet] = list(packets)
        if not burst:
            return iter(())
        offs, total = [], 0
        for p in burst:
            total += A.HEADROOM
            offs.append(total)
            total = (total + len(p.frame) + 15) & ~15
        buf = np.zeros(total + 16, dtype=np.uint8)
        inp = np.zeros(len(burst), dtype=A.PKT_IN)
        for i, p in enumerate(burst):
            buf[offs[i]:offs[i] + len(p.frame)] = np.frombuffer(p.frame, dtype=np.uint8)
            inp[i] = (offs[i], len(p.frame), A.IN_SEEDED_OVERLAY if p.seeded_overlay else 0,
                      p.iif, p.src_vni)
        out = self.process_arrays(buf, inp)
        for i, p in enumerate(burst):
            r = out[i]
            d = int(r["done"])
            p.done = A.DONE_NAMES[d] if d < A.DONE_COUNT else None
            p.meta_flags = int(r["meta_flags"])
            p.oif = int(r["oif"]) or None
            p.dst_vni = int(r["dst_vni"]) or None
            p.fib_entry = None if r["fib_entry"] == 0xFFFFFFFF else int(r["fib_entry"])
            p.acl_rule = None if r["acl_rule"] == 0xFFFFFFFF else int(r["acl_rule"])
            pm = int(r["pm_flags"])
            p.vrf = int(r["vrf"]) if pm & A.PM_HAS_VRF else None
            p.nh_addr = A.nh_text(r) if pm & A.PM_HAS_NH else None
            p.dscp = int(r["dscp"]) if pm & A.PM_HAS_DSCP else None
            p.ecn = int(r["ecn"]) if pm & A.PM_HAS_DSCP else None
            p.flow_ref = int(r["flow_ref"])
            if d == A.DONE["Delivered"]:
                p.frame = bytes(buf[r["off"]:r["off"] + r["len"]])
        return iter(burst)

    def set_host_path(self, mode: int) -> None:
        """dp_ctx_set_option(DP_OPT_HOST_PATH): A.HOST_AUTO / HOST_COPY / HOST_ZERO_COPY."""
        A.check(self.lib.dp_ctx_set_option(self.ctx, A.OPT_HOST_PATH, mode), "dp_ctx_set_option",
                self.lib)

    def set_option(self, option: int, value: int) -> None:
        """dp_ctx_set_option (A.OPT_HOST_PATH, A.OPT_CLOCK: the flow clock in ns)."""
        A.check(self.lib.dp_ctx_set_option(self.ctx, option, value), "dp_ctx_set_option", self.lib)

    def set_clock(self, now_ns: int) -> None:
        """Instant::now() for the bursts that follow (DP_OPT_CLOCK): the expiry
        port forwarding gives the flows it creates and refreshes."""
        self.set_option(A.OPT_CLOCK, now_ns)

    def process_arrays(self, buf: np.ndarray, inp: np.ndarray,
                       stats: Optional[np.ndarray] = None,
                       out: Optional[np.ndarray] = None,
                       meta: Optional[np.ndarray] = None, with_meta: bool = True) -> np.ndarray:
        """Host-origin burst, in place (dp_process_burst).  Returns PKT_RES
        records (dp_pkt_out_t + dp_pkt_meta_t) -- or, with with_meta=False,
        the dp_pkt_out_t array alone (no meta array passed to the path)."""
        if out is None:
            out = np.zeros(len(inp), dtype=A.PKT_OUT)
        if meta is None and with_meta:
            meta = np.zeros(len(inp), dtype=A.PKT_META)
        sp = stats.ctypes.data if stats is not None else None
        A.check(self.lib.dp_process_burst(self.ctx, buf.ctypes.data, buf.nbytes, inp.ctypes.data,
                                          out.ctypes.data,
                                          meta.ctypes.data if meta is not None else None,
                                          len(inp), sp),
                "dp_process_burst", self.lib)
        return A.join_results(out, meta) if meta is not None else out

    def attach_flows(self, flow_table) -> None:
        """FlowLookup::new(name, flow_table) (flow-entry/src/flow_table/nf_lookup.rs:24-32):
        this context's pipeline consults `flow_table` (a dataplane_amd.flows.FlowTable);
        None detaches it (an empty flow table)."""
        A.check(self.lib.dp_ctx_attach_flow_table(self.ctx, flow_table.h if flow_table else None),
                "dp_ctx_attach_flow_table", self.lib)

    def process_mbufs(self, pool_base: int, pool_bytes: int, mbufs: np.ndarray,
                      port_ifindex: Optional[np.ndarray] = None,
                      stats: Optional[np.ndarray] = None, layout=None) -> np.ndarray:
        """An rx burst of rte_mbufs (addresses in `mbufs`) through the path in
        their pinned, device-mapped mempool region (dp_process_mbufs): the
        delivered mbufs hold their serialized frames, ready for tx."""
        mbufs = np.ascontiguousarray(mbufs, dtype=np.uint64)
        out = np.zeros(len(mbufs), dtype=A.PKT_OUT)
        meta = np.zeros(len(mbufs), dtype=A.PKT_META)
        pif = None if port_ifindex is None else np.ascontiguousarray(port_ifindex, dtype=np.uint32)
        A.check(self.lib.dp_process_mbufs(self.ctx, pool_base, pool_bytes, mbufs.ctypes.data,
                                          len(mbufs), C.byref(layout or A.MBUF_LAYOUT_DPDK),
                                          pif.ctypes.data if pif is not None else None,
                                          len(pif) if pif is not None else 0, out.ctypes.data,
                                          meta.ctypes.data,
                                          stats.ctypes.data if stats is not None else None),
                "dp_process_mbufs", self.lib)
        return A.join_results(out, meta)

    def process_device(self, dev_buf: int, buf_bytes: int, dev_in: int, dev_out: int, n: int,
                       dev_stats: Optional[int] = None, stream: Optional[int] = None,
                       dev_meta: Optional[int] = None) -> None:
        """Device-resident burst (dp_process_burst_device): raw device pointers;
        dev_meta (dp_pkt_meta_t[n]) is optional."""
        A.check(self.lib.dp_process_burst_device(self.ctx, dev_buf, buf_bytes, dev_in, dev_out,
                                                 dev_meta, n, dev_stats, stream),
                "dp_process_burst_device", self.lib)

    @staticmethod
    def process_sharded(nfs: List["GpuPathNf"], buf: np.ndarray, inp: np.ndarray,
                        stats: Optional[np.ndarray] = None) -> np.ndarray:
        """Host-origin burst split over several contexts / GPUs
        (dp_process_burst_sharded): contiguous shards of whole packets, one
        per context, copied and processed concurrently."""
        out = np.zeros(len(inp), dtype=A.PKT_OUT)
        meta = np.zeros(len(inp), dtype=A.PKT_META)
        ctxs = (C.c_void_p * len(nfs))(*[nf.ctx for nf in nfs])
        lib = nfs[0].lib
        sp = stats.ctypes.data if stats is not None else None
        A.check(lib.dp_process_burst_sharded(ctxs, len(nfs), buf.ctypes.data, buf.nbytes,
                                             inp.ctypes.data, out.ctypes.data, meta.ctypes.data,
                                             len(inp), sp),
                "dp_process_burst_sharded", lib)
        return A.join_results(out, meta)

    def synchronize(self) -> None:
        A.check(self.lib.dp_ctx_synchronize(self.ctx), "dp_ctx_synchronize", self.lib)

    def device_table_bytes(self) -> int:
        return int(self.lib.dp_tables_device_bytes(self.ctx))

    def acl_classify(self, keys: np.ndarray) -> np.ndarray:
        """The ACL classifier alone (dp_acl_classify): A.ACL_KEY records ->
        A.ACL_RESULT records (the batch Lookup<K, A> of the reference's
        DpdkAclLookup, acl/src/dpdk/lookup.rs:112-155)."""
        keys = np.ascontiguousarray(np.atleast_1d(keys), dtype=A.ACL_KEY)
        out = np.zeros(len(keys), dtype=A.ACL_RESULT)
        A.check(self.lib.dp_acl_classify(self.ctx, keys.ctypes.data, out.ctypes.data, len(keys)),
                "dp_acl_classify", self.lib)
        return out

    def acl_classify_match(self, match: np.ndarray, key_size: int, stride: int = 0) -> np.ndarray:
        """The same over the reference's own key bytes (dp_acl_classify_match):
        AclKey::as_key() output, key_size 21 (v4) or 45 (v6), keys `stride`
        bytes apart (default: packed)."""
        match = np.ascontiguousarray(match, dtype=np.uint8).reshape(-1)
        stride = stride or key_size
        n = len(match) // stride if len(match) >= key_size else 0
        if n and (n - 1) * stride + key_size > len(match):
            n -= 1
        out = np.zeros(n, dtype=A.ACL_RESULT)
        A.check(self.lib.dp_acl_classify_match(self.ctx, match.ctypes.data, key_size, stride, n,
                                               out.ctypes.data), "dp_acl_classify_match", self.lib)
        return out

    def ff_classify(self, inputs: np.ndarray) -> np.ndarray:
        """The flow-filter classifier alone (dp_ff_classify): A.FF_INPUT
        records (LookupInput) -> A.FF_RESULT records (LookupResult) --
        FlowFilterContext::lookup_batch, flow-filter/src/context/tables.rs:800-848."""
        inputs = np.ascontiguousarray(np.atleast_1d(inputs), dtype=A.FF_INPUT)
        out = np.zeros(len(inputs), dtype=A.FF_RESULT)
        A.check(self.lib.dp_ff_classify(self.ctx, inputs.ctypes.data, out.ctypes.data, len(inputs)),
                "dp_ff_classify", self.lib)
        return out

    def ff_classify_match(self, table: int, match: np.ndarray, key_size: int, stride: int = 0) -> np.ndarray:
        """One table alone over the reference's key bytes (dp_ff_classify_match):
        RemoteKey::as_key() (table A.FF_REMOTE, 15 / 27 bytes) or LocalKey::as_key()
        (A.FF_LOCAL, 16 / 28 bytes), keys `stride` bytes apart (default: packed)."""
        match = np.ascontiguousarray(match, dtype=np.uint8).reshape(-1)
        stride = stride or key_size
        n = len(match) // stride if len(match) >= key_size else 0
        if n and (n - 1) * stride + key_size > len(match):
            n -= 1
        out = np.zeros(n, dtype=A.FF_RESULT)
        A.check(self.lib.dp_ff_classify_match(self.ctx, table, match.ctypes.data, key_size, stride, n,
                                              out.ctypes.data), "dp_ff_classify_match", self.lib)
        return out

    def close(self) -> None:
        if self.ctx:
            self.lib.dp_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
