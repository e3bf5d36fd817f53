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
    oout = Oracle(w.tables).process(buf, inp, A.PKT_OUT)
    assert out[5]["done"] == A.DONE["InternalFailure"]
    keep = np.arange(len(frames)) != 5
    for k in ("done", "acl", "meta_flags", "oif", "dst_vni", "src_vni", "fib_entry", "acl_rule"):
        bad = np.nonzero((out[k] != oout[k]) & keep)[0]
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
