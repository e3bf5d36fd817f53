"""GPU parity: the HIP path (through the C ABI) against the oracle on the
same seeded bursts.  Bit-exact on metadata and serialized bytes."""
import numpy as np
import pytest

from dataplane_amd import GpuPathNf, _abi as A
from dataplane_amd.nf import Packet
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle

from edgecase import edge_frames, edge_tables, pack_burst
from helpers import compare, hist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nf():
    # torch (plumbing for the device-path test) bundles its own HIP runtime;
    # it must initialise before libdpgpu's runtime claims the device
    import torch
    torch.cuda.init()
    n = GpuPathNf(0)
    yield n
    n.close()


CASES = [(f, "packed") for f in ("auto", "bv", "list")] + [("auto", "dpdk")]


@pytest.mark.parametrize("form,layout", CASES)
@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_gpu_matches_oracle(nf, cfg, form, layout, cls_form):
    """Classifiers built in each form (dpd_debug_set_classifier_form, read at publish), in
    the packed layout and in the DPDK mbuf layout bench.py times."""
    cls_form(A.gpu_lib(), form)
    w = Workload(cfg, 20000, seed=200 + cfg, n_routes_v4=20000, n_routes_v6=8000, n_acl=1000,
                 n_nat=64, tcp_percent=25, layout=layout)
    nf.publish(w.tables)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    stats = np.zeros(A.DONE_COUNT, dtype=np.uint64)
    o_dut = nf.process_arrays(b_dut, w.inp, stats)
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg}")
    h = hist(o_ref)
    assert int(stats.sum()) == w.n
    assert int(stats[A.DONE["Delivered"]]) == h.get("Delivered", 0)


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_gpu_matches_oracle_without_lds_context(nf, cfg):
    """The same through the units that read the context tables from HBM
    (parts 11 / 12, 13 / 14 with v6 windows; an overlay image whose tables
    fit DPD_CTX_MAX runs parts 1 / 2 or 7 / 8, with a per-workgroup LDS copy)."""
    lib = A.gpu_lib()
    w = Workload(cfg, 20000, seed=300 + cfg, n_routes_v4=20000, n_routes_v6=8000, n_acl=1000, n_nat=64,
                 tcp_percent=25)
    nf.publish(w.tables)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    lib.dpf_debug_no_ctx(1)
    try:
        o_dut = nf.process_arrays(b_dut, w.inp)
    finally:
        lib.dpf_debug_no_ctx(0)
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg} without LDS context")


@pytest.fixture(scope="module")
def edge():
    t = edge_tables()
    return t, t.build()


@pytest.mark.parametrize("seed", [11, 12, 13, 14, 15, 16])
def test_gpu_edge_corpus(nf, edge, seed, cls_form):
    """Malformed / boundary frames and every table branch (tests/edgecase.py);
    odd seeds with bit-vector classifiers, even seeds with candidate lists."""
    cls_form(A.gpu_lib(), "bv" if seed % 2 else "list")
    _, tp = edge
    nf.publish(tp)
    buf, inp = pack_burst(edge_frames(20000, seed))
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = nf.process_arrays(b_dut, inp)
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"edge {seed}")


@pytest.mark.parametrize("cfg,layout", [(2, "dpdk"), (2, "packed"), (3, "dpdk"), (4, "dpdk"),
                                        (5, "dpdk")])
def test_gpu_full_size(nf, cfg, layout):
    """BASELINE.json table sizes (1M v4 routes, 200k v6 on C5, 10k ACL rules
    per family, 256 NAT maps) at 1M packets, bit-exact against the oracle run
    on all host cores; the DPDK mbuf layout is the one bench.py times."""
    import os
    w = Workload(cfg, 1_000_000, seed=300 + cfg, tcp_percent=20, layout=layout)
    nf.publish(w.tables)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref, m_ref = np.zeros(w.n, dtype=A.PKT_OUT), np.zeros(w.n, dtype=A.PKT_META)
    orc = Oracle(w.tables)
    orc.process_parallel(b_ref, w.inp, o_ref, threads=max(1, min(16, len(os.sched_getaffinity(0)))),
                         meta=m_ref)
    o_ref = A.join_results(o_ref, m_ref)
    o_dut = nf.process_arrays(b_dut, w.inp)
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg} full")
    assert hist(o_ref).get("Delivered", 0) > w.n // 4


def test_gpu_device_path_and_determinism(nf):
    """dp_process_burst_device on torch-allocated HBM, on a caller stream;
    processing the same pristine burst twice gives identical results."""
    import torch
    w = Workload(2, 50000, seed=77, n_routes_v4=50000, n_acl=2000, n_nat=64, tcp_percent=30)
    nf.publish(w.tables)
    b_ref = w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev)
    outs = []
    for _ in range(2):
        db = torch.from_numpy(w.fresh_buf()).to(dev)
        di = torch.from_numpy(w.inp.view(np.uint8)).to(dev)
        do = torch.zeros(w.n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
        dm = torch.zeros(w.n * A.PKT_META.itemsize, dtype=torch.uint8, device=dev)
        st = torch.zeros(A.DONE_COUNT, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        nf.process_device(db.data_ptr(), db.numel(), di.data_ptr(), do.data_ptr(), w.n,
                          st.data_ptr(), s.cuda_stream, dev_meta=dm.data_ptr())
        s.synchronize()
        o = A.join_results(do.cpu().numpy().view(A.PKT_OUT), dm.cpu().numpy().view(A.PKT_META))
        b = db.cpu().numpy()
        compare(o_ref, b_ref, o, b, w.inp, "device path")
        assert int(st.sum()) == w.n
        outs.append((o, b))
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("mode", ["copy", "zero_copy", "auto"])
def test_gpu_host_paths_pinned(nf, mode):
    """dp_process_burst on pinned host buffers in each host-path mode
    (dp_ctx_set_option): chunked staging copies, and the kernel working on
    the mapped host frames directly.  Same bytes and records either way."""
    import torch
    m = {"copy": A.HOST_COPY, "zero_copy": A.HOST_ZERO_COPY, "auto": A.HOST_AUTO}[mode]
    w = Workload(2, 150000, seed=91, n_routes_v4=50000, n_acl=2000, n_nat=64, tcp_percent=30,
                 layout="dpdk")
    nf.publish(w.tables)
    b_ref = w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)

    def pinned(nbytes):
        return torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy()
    pb = pinned(w.buf.nbytes)
    pb[:] = w.fresh_buf()
    pi = pinned(w.inp.nbytes).view(A.PKT_IN)
    pi[:] = w.inp
    po = pinned(w.n * A.PKT_OUT.itemsize).view(A.PKT_OUT)
    pm = pinned(w.n * A.PKT_META.itemsize).view(A.PKT_META)
    nf.set_host_path(m)
    try:
        o = nf.process_arrays(pb, pi, out=po, meta=pm)
    finally:
        nf.set_host_path(A.HOST_AUTO)
    compare(o_ref, b_ref, o, pb, w.inp, f"host path {mode}")


def test_gpu_zero_copy_rejects_pageable(nf):
    """Forcing zero copy on pageable (unmapped) buffers fails with an error
    instead of falling back silently."""
    w = Workload(1, 1024, seed=3)
    nf.publish(w.tables)
    nf.set_host_path(A.HOST_ZERO_COPY)
    try:
        with pytest.raises(RuntimeError):
            nf.process_arrays(w.fresh_buf(), w.inp)
    finally:
        nf.set_host_path(A.HOST_AUTO)


def test_gpu_republish_and_empty(nf, edge):
    """A burst after dp_tables_publish sees the new generation; n == 0 is a
    no-op; offsets outside the buffer contract are InternalFailure and touch
    nothing."""
    _, tp = edge
    w = Workload(1, 4096, seed=5)
    nf.publish(w.tables)
    g1 = nf.data.genid
    nf.publish(tp)
    assert nf.data.genid != g1
    buf, inp = pack_burst(edge_frames(4096, 21))
    b_ref, b_dut = buf.copy(), buf.copy()
    compare(Oracle(tp).process(b_ref, inp), b_ref, nf.process_arrays(b_dut, inp),
            b_dut, inp, "after republish")
    assert len(nf.process_arrays(buf.copy(), inp[:0])) == 0
    bad = inp[:4].copy()
    bad["off"] = [0, 16, len(buf) - 8, len(buf) + 4096]
    b = buf.copy()
    with pytest.raises(RuntimeError):   # the host path validates the layout
        nf.process_arrays(b, bad)


def test_gpu_known_answers(nf):
    """The reference's KATs (tests/golden/kat.py) through the HIP path."""
    from golden.kat import all_cases, run_case

    def gpu_process(tp, buf, inp):
        nf.publish(tp)
        return nf.process_arrays(buf, inp)
    errs = []
    for case in all_cases():
        errs += run_case(case, gpu_process)
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("name", ["c1", "c2", "c3", "c4", "c5", "edge"])
def test_gpu_golden_vectors(nf, name):
    """The committed golden vectors, byte for byte."""
    from test_golden import load
    keep, tp, z = load(name)
    nf.publish(tp)
    b = z["buf_in"].copy()
    out = nf.process_arrays(b, z["inp"])
    compare(z["out"], z["buf_out"], out, b, z["inp"], f"golden {name} gpu")


@pytest.mark.parametrize("layout", ["packed", "dpdk"])
def test_gpu_sharded_matches_single(nf, layout):
    """dp_process_burst_sharded over three contexts (one per GPU when the
    box has them, else three streams of GPU 0) equals the oracle bit for bit,
    with the DoneReason counts summed."""
    import torch
    ndev = torch.cuda.device_count()
    w = Workload(2, 30001, seed=91, n_routes_v4=20000, n_acl=800, n_nat=32, tcp_percent=25,
                 layout=layout)
    nfs = [GpuPathNf(k % ndev) for k in range(3)]
    try:
        for x in nfs:
            x.publish(w.tables)
        b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
        o_ref = Oracle(w.tables).process(b_ref, w.inp)
        stats = np.zeros(A.DONE_COUNT, dtype=np.uint64)
        o_dut = GpuPathNf.process_sharded(nfs, b_dut, w.inp, stats)
        compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"sharded {layout}")
        assert int(stats.sum()) == w.n
        assert int(stats[A.DONE["Delivered"]]) == hist(o_ref).get("Delivered", 0)
    finally:
        for x in nfs:
            x.close()


def test_gpu_whole_burst_failure_marks_internal_failure(nf):
    """A burst that cannot run marks every packet InternalFailure besides the
    negative status (dpgpu.h conventions): host path with a frame outside the
    buffer, sharded path with overlapping slots, device path with a
    misaligned buffer."""
    import ctypes as C
    import torch
    w = Workload(1, 256, seed=3)
    nf.publish(w.tables)
    lib = A.gpu_lib()
    bad = w.inp.copy()
    bad["off"][7] = w.buf.nbytes + 64
    out = np.zeros(len(bad), dtype=A.PKT_OUT)
    out["done"] = A.DONE["Delivered"]
    b = w.fresh_buf()
    rc = lib.dp_process_burst(nf.ctx, b.ctypes.data, b.nbytes, bad.ctypes.data, out.ctypes.data,
                              None, len(bad), None)
    assert rc < 0 and np.all(out["done"] == A.DONE["InternalFailure"])
    ovl = w.inp.copy()
    ovl["off"][5] = ovl["off"][4] + 8
    out[:] = 0
    out["done"] = A.DONE["Delivered"]
    ctxs = (C.c_void_p * 1)(nf.ctx)
    rc = lib.dp_process_burst_sharded(ctxs, 1, b.ctypes.data, b.nbytes, ovl.ctypes.data,
                                      out.ctypes.data, None, len(ovl), None)
    assert rc < 0 and np.all(out["done"] == A.DONE["InternalFailure"])
    dev = torch.device("cuda", 0)
    db = torch.from_numpy(w.fresh_buf()).to(dev)
    di = torch.from_numpy(w.inp.view(np.uint8)).to(dev)
    do = torch.full((w.n * A.PKT_OUT.itemsize,), 0x1f, dtype=torch.uint8, device=dev)
    rc = lib.dp_process_burst_device(nf.ctx, db.data_ptr() + 1, db.numel() - 1, di.data_ptr(),
                                     do.data_ptr(), None, w.n, None, None)
    nf.synchronize()
    o = do.cpu().numpy().view(A.PKT_OUT)
    assert rc < 0 and np.all(o["done"] == A.DONE["InternalFailure"])
    assert np.array_equal(o["off"], w.inp["off"])


def test_gpu_meta_through_c_abi(nf, edge):
    """ABI v2 through the raw C entry points: dp_process_burst with a
    dp_pkt_meta_t array gives the oracle's PacketMeta fields (VNIs, FIB
    entry, ACL rule, vrf, nh_addr, dscp / ecn, flow ref) bit-exact; without
    one (meta = NULL) the dp_pkt_out_t records and bytes are the same; the
    NetworkFunction adapter (GpuPathNf.process) carries them onto Packets."""
    _, tp = edge
    nf.publish(tp)
    buf, inp = pack_burst(edge_frames(8000, 21))
    b_ref = buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    lib = A.gpu_lib()
    out = np.zeros(len(inp), A.PKT_OUT)
    meta = np.zeros(len(inp), A.PKT_META)
    meta.view(np.uint8)[:] = 0xA5
    b1 = buf.copy()
    assert lib.dp_process_burst(nf.ctx, b1.ctypes.data, b1.nbytes, inp.ctypes.data,
                                out.ctypes.data, meta.ctypes.data, len(inp), None) == 0
    res = A.join_results(out, meta)
    for k in ("dst_vni", "src_vni", "fib_entry", "acl_rule", "vrf", "pm_flags", "dscp", "ecn",
              "nh_family", "nh_addr", "flow_ref"):
        bad = np.nonzero(np.any((res[k] != o_ref[k]).reshape(len(inp), -1), axis=1))[0]
        assert len(bad) == 0, f"{k} differs at {bad[:5]}"
    assert np.all(res["flow_ref"] == np.uint64(A.FLOW_NONE))
    compare(o_ref, b_ref, res, b1, inp, "meta via C-ABI")
    out2 = np.zeros(len(inp), A.PKT_OUT)
    b2 = buf.copy()
    assert lib.dp_process_burst(nf.ctx, b2.ctypes.data, b2.nbytes, inp.ctypes.data,
                                out2.ctypes.data, None, len(inp), None) == 0
    assert np.array_equal(out, out2) and np.array_equal(b1, b2)
    pkts = [Packet(frame=bytes(buf[o:o + n]), iif=int(i), src_vni=int(v),
                   seeded_overlay=bool(f & A.IN_SEEDED_OVERLAY))
            for o, n, f, i, v in zip(inp["off"], inp["len"], inp["flags"], inp["iif"],
                                     inp["src_vni"])]
    got = list(nf.process(pkts))
    pm = o_ref["pm_flags"]
    for j, p in enumerate(got):
        assert p.vrf == (int(o_ref[j]["vrf"]) if pm[j] & A.PM_HAS_VRF else None)
        assert p.nh_addr == (A.nh_text(o_ref[j]) if pm[j] & A.PM_HAS_NH else None)
        assert p.dscp == (int(o_ref[j]["dscp"]) if pm[j] & A.PM_HAS_DSCP else None)
        assert p.done == A.DONE_NAMES[int(o_ref[j]["done"])]


def test_gpu_sharded_full_size_c5(nf):
    """BASELINE config 5 (v4 + v6 mix, 1M v4 + 200k v6 routes, 10k ACL rules
    per family, NAT) at 1M packets through dp_process_burst_sharded, one
    context per visible GPU (at least three, dealt round-robin over the
    devices), bit-exact against the oracle on the host cores."""
    import os
    import torch
    ndev = torch.cuda.device_count()
    w = Workload(5, 1_000_000, seed=505, tcp_percent=20, layout="dpdk")
    nfs = [GpuPathNf(k % ndev) for k in range(max(3, ndev))]
    try:
        for x in nfs:
            x.publish(w.tables)
        b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
        o_ref, m_ref = np.zeros(w.n, dtype=A.PKT_OUT), np.zeros(w.n, dtype=A.PKT_META)
        Oracle(w.tables).process_parallel(b_ref, w.inp, o_ref,
                                          threads=max(1, min(16, len(os.sched_getaffinity(0)))),
                                          meta=m_ref)
        o_ref = A.join_results(o_ref, m_ref)
        stats = np.zeros(A.DONE_COUNT, dtype=np.uint64)
        o_dut = GpuPathNf.process_sharded(nfs, b_dut, w.inp, stats)
        compare(o_ref, b_ref, o_dut, b_dut, w.inp, "C5 sharded full size")
        assert int(stats.sum()) == w.n
        h = hist(o_ref)
        assert int(stats[A.DONE["Delivered"]]) == h.get("Delivered", 0) > w.n // 4
    finally:
        for x in nfs:
            x.close()


def test_gpu_sharded_then_larger_staged_burst():
    """One context first runs a sharded burst (which sizes its device records)
    and then a larger staged-copy burst (pageable buffers): every per-packet
    array of the host paths grows together (dp_runtime.cpp ensure_records), so
    the staged burst never writes past a smaller allocation."""
    w_small = Workload(2, 3000, seed=41, n_routes_v4=5000, n_acl=200, n_nat=16)
    w_big = Workload(2, 40000, seed=42, n_routes_v4=5000, n_acl=200, n_nat=16)
    x = GpuPathNf(0)
    try:
        x.publish(w_small.tables)
        b_ref, b_dut = w_small.fresh_buf(), w_small.fresh_buf()
        compare(Oracle(w_small.tables).process(b_ref, w_small.inp), b_ref,
                GpuPathNf.process_sharded([x], b_dut, w_small.inp), b_dut, w_small.inp, "sharded first")
        x.publish(w_big.tables)
        x.set_host_path(A.HOST_COPY)
        b_ref, b_dut = w_big.fresh_buf(), w_big.fresh_buf()
        compare(Oracle(w_big.tables).process(b_ref, w_big.inp), b_ref,
                x.process_arrays(b_dut, w_big.inp), b_dut, w_big.inp, "staged after sharded")
    finally:
        x.close()
