"""GPU: the flow table (dp_flow_*) and the flows variant of the pipeline
through the C ABI, against the oracle's restatement of the reference
(FlowTable, FlowLookup, the flow-aware FlowFilter / AclFilter /
IcmpErrorHandler branches, the burst order).  Bit-exact."""
import numpy as np
import pytest

from dataplane_amd import GpuPathNf, _abi as A
from dataplane_amd.flows import FlowTable
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle, OracleFlows

from edgecase import pack_burst
from flowgen import frames_of, install, scenario
from golden.flowkat import all_cases, run_case
from helpers import compare
from test_flows import table_semantics

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nf():
    import torch
    torch.cuda.init()
    n = GpuPathNf(0)
    yield n
    n.attach_flows(None)
    n.close()


def run_device(nf, buf, inp, stats=False):
    """One device-resident burst with flow refs out: (out, refs[, stats]);
    `buf` is rewritten in place."""
    import torch
    dev = torch.device("cuda", 0)
    db = torch.from_numpy(buf).to(dev)
    di = torch.from_numpy(inp.view(np.uint8).copy()).to(dev)
    do = torch.zeros(len(inp) * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
    dm = torch.zeros(len(inp) * A.PKT_META.itemsize, dtype=torch.uint8, device=dev)
    st = torch.zeros(A.DONE_COUNT, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    nf.process_device(db.data_ptr(), db.numel(), di.data_ptr(), do.data_ptr(), len(inp),
                      st.data_ptr(), dev_meta=dm.data_ptr())
    nf.synchronize()
    buf[:] = db.cpu().numpy()
    out = A.join_results(do.cpu().numpy().view(A.PKT_OUT), dm.cpu().numpy().view(A.PKT_META))
    refs = out["flow_ref"].copy()
    return (out, refs, st.cpu().numpy().view(np.uint64)) if stats else (out, refs)


class GpuBackend:
    def __init__(self, nf):
        self.nf = nf

    def table(self):
        return FlowTable(0, 1 << 12)

    def process(self, tb, buf, inp, ft):
        self.nf.publish(tb.build())
        self.nf.attach_flows(ft)
        try:
            return run_device(self.nf, buf, inp)
        finally:
            self.nf.attach_flows(None)


def test_gpu_flow_table_semantics(nf):
    # (nf: torch's HIP runtime initialises before libdpgpu's claims the device)
    table_semantics(FlowTable(0, 1 << 10))


def test_gpu_flow_known_answers(nf):
    errs = []
    for case in all_cases():
        errs += run_case(case, GpuBackend(nf))
    assert not errs, "\n".join(errs)


def _ref_map(a, b):
    """Translate refs of table `a` to refs of table `b` by insertion order."""
    return {x: y for x, y in zip(a, b) if x != A.FLOW_NONE}


@pytest.mark.parametrize("full", [False, True], ids=["auto", "full"])
@pytest.mark.parametrize("cfg,seed", [(2, 1), (2, 2), (5, 3)])
def test_gpu_flows_random_bursts(nf, cfg, seed, full):
    """Seeded scenarios (tests/flowgen.py) over a C2-shaped workload, and a
    C5-shaped one (v4 / v6 mix: v6 flow keys, v6 ACL reply path): two bursts
    in a row, then the flow timers; outputs, serialized bytes, flow refs and
    every flow's state equal the oracle's.  auto: the C2 image configures no
    stateful NAT and has no v6 windows, so its bursts run the lean flows
    variant (parts 9 / 10); full: the variant with stateful NAT compiled in."""
    w = Workload(cfg, 6000, seed=seed, n_routes_v4=3000, n_routes_v6=2000 if cfg == 5 else 0,
                 n_acl=400, n_nat=24, tcp_percent=30)
    ora = Oracle(w.tables)
    frames = frames_of(w)
    ob = w.fresh_buf()
    o0 = ora.process(ob, w.inp)
    items, burst = scenario(frames, o0["dst_vni"], genid=1, seed=seed, n_flows=600,
                            vnis=sorted(set(int(v) for v in o0["dst_vni"] if v)))
    if cfg == 5:
        assert sum(int(it[1]["key"]["family"]) == 6 for it in items) > 50
    oft, gft = OracleFlows(), FlowTable(0, 1 << 13)
    orefs, grefs = install(oft, items), install(gft, items)
    g2o = _ref_map(grefs, orefs)
    nf.publish(w.tables)
    nf.attach_flows(gft)
    lib = A.gpu_lib()
    lib.dpf_debug_flows_full(1 if full else 0)
    try:
        for rnd in range(2):
            buf, inp = pack_burst([(f, 1, A.IN_SEEDED_OVERLAY, v) for f, v in burst])
            obuf, gbuf = buf.copy(), buf.copy()
            oout, oref, ost = ora.process_flows(obuf, inp, oft, stats=True)
            gout, gref, gst = run_device(nf, gbuf, inp, stats=True)
            if cfg == 2:
                assert lib.dpf_debug_last_lean() == (0 if full else 1), "flows variant"
            compare(oout, obuf, gout, gbuf, inp, f"flows C{cfg} seed {seed} burst {rnd}")
            mapped = np.array([g2o.get(int(r), A.FLOW_NONE) if int(r) != A.FLOW_NONE else A.FLOW_NONE
                               for r in gref], dtype=np.uint64)
            assert np.array_equal(mapped, oref), f"flow refs differ ({np.count_nonzero(mapped != oref)})"
            assert np.array_equal(gst, ost), "DoneReason histogram"
            assert int((oout["acl"] == 6).sum()) > 0, "no packet took the flow-scope reply path"
            gi, oi = gft.get(grefs), oft.get(orefs)
            for j in range(len(grefs)):
                gone_g, gone_o = gi[j]["ref"] == A.FLOW_NONE, oi[j]["ref"] == A.FLOW_NONE
                assert gone_g == gone_o, f"flow {j} presence"
                if not gone_g:
                    assert gi[j]["status"] == oi[j]["status"], f"flow {j} status (burst {rnd})"
        assert gft.count() == oft.count()
        assert gft.sweep(1 << 62) == oft.sweep(1 << 62)
        assert gft.count() == oft.count()
    finally:
        lib.dpf_debug_flows_full(0)
        nf.attach_flows(None)


def test_gpu_flows_empty_table_matches_no_table(nf):
    """An attached empty flow table changes nothing."""
    w = Workload(2, 4096, seed=5, n_routes_v4=2000, n_acl=300, n_nat=16)
    ft = FlowTable(0, 1 << 8)
    nf.publish(w.tables)
    b0, b1 = w.fresh_buf(), w.fresh_buf()
    out0 = nf.process_arrays(b0, w.inp)
    nf.attach_flows(ft)
    try:
        out1, refs = run_device(nf, b1, w.inp)
    finally:
        nf.attach_flows(None)
    compare(out0, b0, out1, b1, w.inp, "empty flow table")
    assert (refs == np.uint64(A.FLOW_NONE)).all()


def test_gpu_flows_full_size(nf):
    """BASELINE.json's C2 tables (1M routes, 10k ACL rules, NAT) with a
    flow table of ~250k established flows over a 500k-packet burst: every
    output, byte, flow ref and flow state equals the oracle's."""
    from dataplane_amd.flows import burst_request_flows
    w = Workload(2, 500_000, seed=9)
    ora = Oracle(w.tables)
    nf.publish(w.tables)
    o0 = nf.process_arrays(w.fresh_buf(), w.inp)   # each packet's flow-filter verdict
    fl = burst_request_flows(w.buf, w.inp, np.arange(0, w.n, 2), o0["dst_vni"], genid=1)
    # a tenth of them from another generation, a tenth towards another VPC
    fl["genid"][::10] = 0
    fl["dst_vni"][5::10] = np.roll(fl["dst_vni"], 1)[5::10]
    oft, gft = OracleFlows(), FlowTable(0, 1 << 20)
    oref, ores = oft.insert(fl)
    gref, gres = gft.insert(fl)
    assert np.array_equal(ores, gres) and (gres == A.FLOW_INSERTED).all()
    g2o = _ref_map(gref, oref)
    nf.attach_flows(gft)
    try:
        obuf, gbuf = w.fresh_buf(), w.fresh_buf()
        oout, orf = ora.process_flows(obuf, w.inp, oft)
        gout, grf = run_device(nf, gbuf, w.inp)
    finally:
        nf.attach_flows(None)
    compare(oout, obuf, gout, gbuf, w.inp, "flows full size")
    mapped = np.array([g2o.get(int(r), A.FLOW_NONE) if int(r) != A.FLOW_NONE else A.FLOW_NONE
                       for r in grf], dtype=np.uint64)
    assert np.array_equal(mapped, orf)
    assert int((orf != np.uint64(A.FLOW_NONE)).sum()) >= len(fl)
    gi, oi = gft.get(gref), oft.get(oref)
    assert np.array_equal(gi["status"], oi["status"])
    assert gft.count() == oft.count()


def test_gpu_flows_host_origin(nf):
    """With a flow table attached, the host-origin entry (dp_process_burst:
    the burst is one launch, never chunked, since flow-filter invalidations
    must reach every later packet of the burst) matches the oracle on a burst
    larger than the host path's chunk; the sharded entry refuses contexts
    attached to different flow tables."""
    from dataplane_amd.flows import burst_request_flows
    w = Workload(2, 150_000, seed=11, n_routes_v4=5000, n_acl=500, n_nat=24, tcp_percent=30)
    ora = Oracle(w.tables)
    nf.publish(w.tables)
    o0 = nf.process_arrays(w.fresh_buf(), w.inp)
    fl = burst_request_flows(w.buf, w.inp, np.arange(0, w.n, 3), o0["dst_vni"], genid=1)
    fl["genid"][::7] = 0
    oft, gft = OracleFlows(), FlowTable(0, 1 << 18)
    oref, _ = oft.insert(fl)
    gref, _ = gft.insert(fl)
    nf.attach_flows(gft)
    try:
        obuf, hbuf = w.fresh_buf(), w.fresh_buf()
        oout, _ = ora.process_flows(obuf, w.inp, oft)
        hout = nf.process_arrays(hbuf, w.inp)
        other = GpuPathNf(0)
        try:
            with pytest.raises(RuntimeError):
                GpuPathNf.process_sharded([nf, other], w.fresh_buf(), w.inp)
        finally:
            other.close()
    finally:
        nf.attach_flows(None)
    compare(oout, obuf, hout, hbuf, w.inp, "flows host-origin")
    assert np.array_equal(gft.get(gref)["status"], oft.get(oref)["status"])
    assert gft.count() == oft.count()


def test_gpu_flows_two_contexts_one_table(nf):
    """Two worker contexts attached to one flow table (one
    table per device, every worker's context attached) run flows bursts on
    their own streams, launched back to back: the table orders them (the
    burst-local invalidation marks live in the shared slots), so outputs and
    flow states equal the oracle's two bursts run one after the other."""
    import torch
    w = Workload(2, 8000, seed=21, n_routes_v4=3000, n_acl=400, n_nat=24, tcp_percent=30)
    ora = Oracle(w.tables)
    frames = frames_of(w)
    o0 = ora.process(w.fresh_buf(), w.inp)
    items, burst = scenario(frames, o0["dst_vni"], genid=1, seed=21, n_flows=700,
                            vnis=sorted(set(int(v) for v in o0["dst_vni"] if v)))
    oft, gft = OracleFlows(), FlowTable(0, 1 << 13)
    orefs, grefs = install(oft, items), install(gft, items)
    half = len(burst) // 2
    bursts = [pack_burst([(f, 1, A.IN_SEEDED_OVERLAY, v) for f, v in part])
              for part in (burst[:half], burst[half:])]
    nf2 = GpuPathNf(0)
    dev = torch.device("cuda", 0)
    try:
        for x in (nf, nf2):
            x.publish(w.tables)
            x.attach_flows(gft)
        streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
        dbufs, dins, douts = [], [], []
        for buf, inp in bursts:
            dbufs.append(torch.from_numpy(buf.copy()).to(dev))
            dins.append(torch.from_numpy(inp.view(np.uint8).copy()).to(dev))
            douts.append(torch.zeros(len(inp) * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev))
        torch.cuda.synchronize(dev)
        for k, x in enumerate((nf, nf2)):
            x.process_device(dbufs[k].data_ptr(), dbufs[k].numel(), dins[k].data_ptr(),
                             douts[k].data_ptr(), len(bursts[k][1]), None, streams[k].cuda_stream)
        torch.cuda.synchronize(dev)
        for k, (buf, inp) in enumerate(bursts):
            obuf = buf.copy()
            oout, _ = ora.process_flows(obuf, inp, oft)
            gbuf = dbufs[k].cpu().numpy()
            gout = douts[k].cpu().numpy().view(A.PKT_OUT)
            compare(oout, obuf, gout, gbuf, inp, f"two contexts, burst {k}")
        gi, oi = gft.get(grefs), oft.get(orefs)
        assert np.array_equal(gi["ref"] == A.FLOW_NONE, oi["ref"] == A.FLOW_NONE)
        live = gi["ref"] != A.FLOW_NONE
        assert np.array_equal(gi["status"][live], oi["status"][live])
    finally:
        for x in (nf, nf2):
            x.attach_flows(None)
        nf2.close()


def test_gpu_flow_table_churn(nf):
    """Insert / timer-sweep cycles (tombstones): removals leave no
    unbounded tombstone build-up -- runs of tombstones that end a cluster are
    reclaimed, lookups probe at most max_probe + 1 slots -- and every lookup
    stays right: live flows are found, expired ones are not."""
    from dataplane_amd.flows import flow_key, make_flow
    rng = np.random.default_rng(5)
    slots = 1 << 12
    gft = FlowTable(0, slots)
    gft.set_capacity(3000)           # above the 2100 flows a cycle holds before its sweep
    prev = None
    try:
        for cyc in range(1, 41):
            fl = np.zeros(1400, A.FLOW)
            for i in range(len(fl)):
                a = rng.integers(1, 2**31, size=2)
                fl[i] = make_flow(flow_key(7, int(a[0]), int(a[1]), A.FLOW_UDP,
                                           int(rng.integers(1, 65535)), int(rng.integers(1, 65535))),
                                  dst_vni=9, genid=1, expires_at=cyc + (i % 2))
            refs, res = gft.insert(fl)
            assert (res == A.FLOW_INSERTED).all()
            removed = gft.sweep(cyc)                  # this cycle's even flows, last cycle's odd ones
            st = gft.debug_stats()
            assert st["full"] == gft.count()[0]
            assert st["max_probe"] <= 64, st
            assert st["empty"] >= slots // 4, st      # without reclamation: 0 by cycle 18
            found = gft.lookup(fl["key"])
            live = (np.arange(len(fl)) % 2) == 1
            assert (found["ref"][live] != A.FLOW_NONE).all()
            assert (found["ref"][~live] == A.FLOW_NONE).all()
            if prev is not None:
                assert (gft.lookup(prev["key"])["ref"] == A.FLOW_NONE).all()
                assert removed == len(fl) // 2 + len(prev) // 2
            prev = fl
    finally:
        gft.close()
