"""DPDK rx/tx burst glue: the mbuf <-> burst-record
translation of libdpgpu (host-only functions, no GPU), against rte_mbuf
semantics (Mbuf::raw_data, rte_pktmbuf_prepend / _adj; dpdk/src/mem.rs)."""
import ctypes as C

import numpy as np

from dataplane_amd import _abi as A
from mbufpool import HDR, HEADROOM, FakeMempool


def burst_in(pool, mbufs, port_ifindex=None):
    lib = A.gpu_lib()
    inp = np.zeros(len(mbufs), A.PKT_IN)
    pif = None if port_ifindex is None else np.ascontiguousarray(port_ifindex, np.uint32)
    assert lib.dp_mbuf_burst_in(pool.base, pool.mem.nbytes, mbufs.ctypes.data, len(mbufs),
                                C.byref(A.MBUF_LAYOUT_DPDK),
                                pif.ctypes.data if pif is not None else None,
                                len(pif) if pif is not None else 0, inp.ctypes.data) == 0
    return inp


def test_mbuf_burst_records():
    pool = FakeMempool(np.zeros(FakeMempool.bytes_for(8), np.uint8))
    frames = [bytes([i]) * (60 + i) for i in range(6)]
    mbufs = pool.load(frames, ports=[0, 1, 2, 1, 0, 3])
    inp = burst_in(pool, mbufs, port_ifindex=[10, 11, 12])
    for i, f in enumerate(frames):
        assert inp[i]["off"] == i * (pool.addr(1) - pool.addr(0)) + HDR + HEADROOM
        assert inp[i]["len"] == len(f)
        assert bytes(pool.mem[inp[i]["off"]:inp[i]["off"] + len(f)]) == f
    assert list(inp["iif"]) == [10, 11, 12, 11, 10, 0]   # port 3: beyond the map
    assert list(burst_in(pool, mbufs)["iif"]) == [0, 1, 2, 1, 0, 3]  # no map: the port


def test_mbuf_records_outside_the_contract():
    pool = FakeMempool(np.zeros(FakeMempool.bytes_for(4), np.uint8))
    mbufs = pool.load([b"\x01" * 60] * 4, ports=[0] * 4)
    pool.set_field(1, "data_off", 64)                       # headroom < DP_HEADROOM
    pool.set_field(2, "buf_addr", pool.base - 4096)         # outside the region
    pool.set_field(3, "data_len", 4000)                     # runs past the region's end
    inp = burst_in(pool, mbufs)
    assert inp[0]["off"] >= A.HEADROOM
    for i in (1, 2, 3):
        assert inp[i]["off"] == 0 and inp[i]["len"] == 0


def test_mbuf_burst_results():
    """Delivered mbufs describe the serialized frame (grown into the headroom,
    or shrunk); other mbufs are left as received."""
    lib = A.gpu_lib()
    pool = FakeMempool(np.zeros(FakeMempool.bytes_for(4), np.uint8))
    mbufs = pool.load([b"\x02" * 110, b"\x03" * 60, b"\x04" * 60, b"\x05" * 64], ports=[0] * 4)
    inp = burst_in(pool, mbufs)
    out = np.zeros(4, A.PKT_OUT)
    out["done"] = [A.DONE["Delivered"], A.DONE["Delivered"], A.DONE["AclDropped"], A.DONE["Delivered"]]
    out["off"] = inp["off"] + np.array([50, -50, 0, 0])      # decap / encap / - / in place
    out["len"] = [60, 110, 60, 64]
    assert lib.dp_mbuf_burst_out(mbufs.ctypes.data, 4, C.byref(A.MBUF_LAYOUT_DPDK), inp.ctypes.data,
                                 out.ctypes.data) == 0
    assert (pool.field(0, "data_off"), pool.field(0, "data_len"), pool.field(0, "pkt_len")) == (HEADROOM + 50, 60, 60)
    assert (pool.field(1, "data_off"), pool.field(1, "data_len"), pool.field(1, "pkt_len")) == (HEADROOM - 50, 110, 110)
    assert (pool.field(2, "data_off"), pool.field(2, "data_len")) == (HEADROOM, 60)
    assert (pool.field(3, "data_off"), pool.field(3, "data_len")) == (HEADROOM, 64)


def test_mbuf_frame_at_pool_tail_fails_alone():
    """A frame whose end lies inside the pool but whose end rounded up to 16
    bytes (the kernel's 16-byte staging) does not fit gets its own failure record;
    the other mbufs keep theirs (no whole-burst DP_EINVAL later)."""
    lib = A.gpu_lib()
    pool = FakeMempool(np.zeros(FakeMempool.bytes_for(2), np.uint8))
    mbufs = pool.load([b"\x01" * 60, b"\x02" * 61], ports=[0, 0])
    full = burst_in(pool, mbufs)
    end = int(full[1]["off"]) + 61                    # the last frame's exact end
    assert end % 16 != 0
    inp = np.zeros(2, A.PKT_IN)
    assert lib.dp_mbuf_burst_in(pool.base, end, mbufs.ctypes.data, 2, C.byref(A.MBUF_LAYOUT_DPDK),
                                None, 0, inp.ctypes.data) == 0
    assert inp[0]["off"] == full[0]["off"] and inp[0]["len"] == 60
    assert inp[1]["off"] == 0 and inp[1]["len"] == 0
    assert lib.dp_mbuf_burst_in(pool.base, (end + 15) & ~15, mbufs.ctypes.data, 2,
                                C.byref(A.MBUF_LAYOUT_DPDK), None, 0, inp.ctypes.data) == 0
    assert inp[1]["off"] == full[1]["off"]
