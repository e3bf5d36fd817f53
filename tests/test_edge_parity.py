"""CPU: edge-case corpus (tests/edgecase.py) -- the kernel's per-packet code
compiled for the host against the oracle, bit-exact, plus coverage checks
that the corpus really reaches the branches it is meant to."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from oracle.pyoracle import Oracle
import pyemu

from edgecase import edge_frames, edge_tables, pack_burst
from helpers import compare, hist


@pytest.fixture(scope="module")
def tables():
    t = edge_tables()
    return t, t.build()


@pytest.mark.parametrize("form", ["auto", "bv", "list"])
@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_edge_emu_matches_oracle(tables, seed, form, cls_form):
    cls_form(pyemu.lib(), form)
    _, tp = tables
    frames = edge_frames(4000, seed)
    buf, inp = pack_burst(frames)
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = pyemu.process(tp, b_dut, inp)
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"edge seed {seed}")


@pytest.mark.parametrize("seed", [5, 6])
def test_edge_small_window_matches_oracle(tables, seed):
    """A 32-byte LDS header window: every header byte past it is read from
    (and relocated within) the burst buffer."""
    _, tp = tables
    buf, inp = pack_burst(edge_frames(4000, seed))
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = pyemu.process(tp, b_dut, inp, variant="w32")
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"edge w32 seed {seed}")


@pytest.mark.parametrize("cfg", [3, 4, 5])
def test_workload_small_window_matches_oracle(cfg):
    from dataplane_amd.workload import Workload
    w = Workload(cfg, 2000, seed=900 + cfg, n_routes_v4=2000, n_routes_v6=1000, n_acl=200,
                 n_nat=32, tcp_percent=30)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    o_dut = pyemu.process(w.tables, b_dut, w.inp, variant="w32")
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg} w32")


def test_edge_corpus_coverage(tables):
    """The corpus must reach (almost) every DoneReason the path can produce."""
    _, tp = tables
    frames = edge_frames(16000, 99)
    buf, inp = pack_burst(frames)
    out = Oracle(tp).process(buf, inp)
    h = hist(out)
    must = ["InterfaceUnknown", "InterfaceDetached", "InterfaceAdmDown", "InterfaceOperDown",
            "InterfaceUnsupported", "NotEthernet", "Unhandled", "MacNotForUs", "InvalidDstMac",
            "NotIp", "RouteFailure", "RouteDrop", "HopLimitExceeded", "MissL2resolution",
            "VxlanDecapFailure", "VxlanEncapFailure", "Filtered", "AclDropped", "Unroutable",
            "InternalFailure", "Local", "Delivered"]
    missing = [m for m in must if m not in h]
    assert not missing, f"corpus misses {missing}: {h}"
    f = out["meta_flags"]
    for flag in ("NATTED_SRC", "NATTED_DST", "IS_OVERLAY", "REQ_STATIC_NAT_SRC",
                 "REQ_STATIC_NAT_DST", "IS_L2_BCAST"):
        assert np.any(f & A.META[flag]), flag
    assert set(np.unique(out["acl"])) >= {0, 1, 2, 3, 4, 5}
    # dp_pkt_meta_t: every Option<> of PacketMeta the path sets is reached
    pm = out["pm_flags"]
    for flag in (A.PM_HAS_VRF, A.PM_HAS_NH, A.PM_HAS_DSCP):
        assert np.any(pm & flag), flag
    assert set(np.unique(out["nh_family"][(pm & A.PM_HAS_NH) != 0])) == {4, 6}
    assert len(np.unique(out["dscp"][(pm & A.PM_HAS_DSCP) != 0])) > 4


@pytest.mark.parametrize("form", ["bv", "list"])
def test_edge_outline_matches_oracle(tables, form, cls_form):
    """Every device function kept out of line (tests/emu libdpemu_outline.so:
    -fno-inline, DP_COLD honoured): the by-reference call shape of the GPU's
    noinline functions (classify_bv) runs under the CPU suite too."""
    cls_form(pyemu.lib("outline"), form)
    _, tp = tables
    buf, inp = pack_burst(edge_frames(3000, 7))
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = pyemu.process(tp, b_dut, inp, variant="outline")
    if form == "bv":
        assert pyemu.classifier_forms("outline")[0] > 0
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"edge outline {form}")


@pytest.mark.parametrize("cfg", [2, 5])
def test_workload_outline_matches_oracle(cfg, cls_form):
    from dataplane_amd.workload import Workload
    cls_form(pyemu.lib("outline"), "bv")
    w = Workload(cfg, 2000, seed=950 + cfg, n_routes_v4=2000, n_routes_v6=1000, n_acl=200,
                 n_nat=32, tcp_percent=30)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    o_dut = pyemu.process(w.tables, b_dut, w.inp, variant="outline")
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg} outline")
