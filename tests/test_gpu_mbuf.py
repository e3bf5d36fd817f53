"""GPU: an rx burst of rte_mbufs through dp_process_mbufs (the DPDK glue,
SURVEY.md §8f rank 2) -- frames processed in place in a pinned, mapped
mempool region -- against the oracle on the same frames."""
import numpy as np
import pytest

from dataplane_amd import GpuPathNf, _abi as A
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle

from edgecase import pack_burst
from flowgen import frames_of
from helpers import field_diff
from mbufpool import HEADROOM, FakeMempool

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nf():
    import torch
    torch.cuda.init()
    n = GpuPathNf(0)
    yield n
    n.close()


def pinned(nbytes):
    import torch
    return torch.zeros(nbytes, dtype=torch.uint8).pin_memory().numpy()


@pytest.mark.parametrize("cfg", [1, 4])
def test_gpu_mbuf_burst(nf, cfg):
    """C1 (underlay) and C4 (VXLAN decap, NAT, re-encap)."""
    w = Workload(cfg, 3000, seed=7, n_routes_v4=2000, n_acl=200, n_nat=16)
    frames = [f for f, _ in frames_of(w)]
    ports = w.inp["iif"]
    pool = FakeMempool(pinned(FakeMempool.bytes_for(len(frames) + 1)))
    mbufs = pool.load(frames, ports)
    pool.set_field(5, "data_off", 64)   # one mbuf outside the headroom contract
    nf.publish(w.tables)
    st = np.zeros(A.DONE_COUNT, np.uint64)
    out = nf.process_mbufs(pool.base, pool.mem.nbytes, mbufs, stats=st)
    buf, inp = pack_burst([(f, int(p), 0, 0) for f, p in zip(frames, ports)])
    oout = Oracle(w.tables).process(buf, inp)
    assert out[5]["done"] == A.DONE["InternalFailure"]
    keep = np.arange(len(frames)) != 5
    for k in ("done", "acl", "meta_flags", "oif", "dst_vni", "src_vni", "fib_entry", "acl_rule",
              "vrf", "pm_flags", "dscp", "ecn", "nh_family", "nh_addr"):
        bad = np.nonzero(field_diff(out, oout, k) & keep)[0]
        assert len(bad) == 0, f"{k} differs at {bad[:5]}: {out[bad[:1]]} vs {oout[bad[:1]]}"
    deliv = np.nonzero((oout["done"] == A.DONE["Delivered"]) & keep)[0]
    assert len(deliv) > len(frames) // 2
    for i in deliv:
        o, ln = int(oout[i]["off"]), int(oout[i]["len"])
        assert pool.frame(int(i)) == buf[o:o + ln].tobytes(), f"packet {i} frame"
        assert pool.field(int(i), "data_off") - HEADROOM == o - int(inp[i]["off"])
        assert pool.field(int(i), "pkt_len") == ln
    assert int(st.sum()) == len(frames) and int(st[A.DONE["Delivered"]]) == len(deliv)


def test_gpu_mbuf_pool_must_be_mapped(nf):
    w = Workload(1, 64, seed=3, n_routes_v4=100)
    frames = [f for f, _ in frames_of(w)]
    pool = FakeMempool(np.zeros(FakeMempool.bytes_for(len(frames)), np.uint8))
    mbufs = pool.load(frames, w.inp["iif"])
    nf.publish(w.tables)
    with pytest.raises(RuntimeError):
        nf.process_mbufs(pool.base, pool.mem.nbytes, mbufs)


def test_gpu_mbuf_burst_with_flows(nf):
    """C4 through the DPDK glue with a flow table attached: FlowLookup runs on
    the decapsulated overlay packets (flows keyed by the inner 5-tuple and the
    VXLAN VNI, half of them from a stale generation, a quarter towards an
    unknown VPC); outputs, frames and flow states equal the oracle's."""
    from dataplane_amd.flows import FlowTable, make_flow
    from oracle.pyoracle import OracleFlows
    from flowgen import frame_key
    w = Workload(4, 3000, seed=8, n_routes_v4=2000, n_acl=200, n_nat=16)
    frames = [f for f, _ in frames_of(w)]
    ports = w.inp["iif"]
    buf, inp = pack_burst([(f, int(p), 0, 0) for f, p in zip(frames, ports)])
    ora = Oracle(w.tables)
    o0 = ora.process(buf.copy(), inp)
    genid = int(w.tables.contents.genid)
    vnis = sorted(set(int(v) for v in o0["dst_vni"] if v))
    fls, seen = [], set()
    for i in range(0, len(frames), 2):
        f = frames[i]
        if len(f) < 84 or f[12:14] != b"\x08\x00" or f[23] != 17 or f[36:38] != b"\x12\xb5":
            continue
        k = frame_key(f[50:], int.from_bytes(f[46:49], "big"))
        if k is None or not o0[i]["dst_vni"] or k.tobytes() in seen:
            continue
        seen.add(k.tobytes())
        d = int(o0[i]["dst_vni"])
        if len(fls) % 4 == 2:            # a flow towards a VPC the tables do not know
            d = max(vnis) + 17
        fls.append(make_flow(k, d, A.FLOW_INITIATOR, genid=genid - (len(fls) & 1)))
    assert len(fls) > 300
    fl = np.array(fls, dtype=A.FLOW)
    oft, gft = OracleFlows(), FlowTable(0, 1 << 13)
    oref, _ = oft.insert(fl)
    gref, _ = gft.insert(fl)
    oout, _ = ora.process_flows(buf, inp, oft)
    pool = FakeMempool(pinned(FakeMempool.bytes_for(len(frames) + 1)))
    mbufs = pool.load(frames, ports)
    nf.publish(w.tables)
    nf.attach_flows(gft)
    try:
        out = nf.process_mbufs(pool.base, pool.mem.nbytes, mbufs)
    finally:
        nf.attach_flows(None)
    for k in ("done", "acl", "meta_flags", "oif", "dst_vni", "src_vni", "fib_entry", "acl_rule",
              "vrf", "pm_flags", "dscp", "ecn", "nh_family", "nh_addr"):
        bad = np.nonzero(field_diff(out, oout, k))[0]
        assert len(bad) == 0, f"{k} differs at {bad[:5]}"
    for i in np.nonzero(oout["done"] == A.DONE["Delivered"])[0]:
        o, ln = int(oout[i]["off"]), int(oout[i]["len"])
        assert pool.frame(int(i)) == buf[o:o + ln].tobytes(), f"packet {i} frame"
    assert np.array_equal(gft.get(gref)["status"], oft.get(oref)["status"])
    assert gft.count() == oft.count()
