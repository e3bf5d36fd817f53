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


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_edge_emu_matches_oracle(tables, seed):
    _, tp = tables
    frames = edge_frames(4000, seed)
    buf, inp = pack_burst(frames)
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp, A.PKT_OUT)
    o_dut = pyemu.process(tp, b_dut, inp, A.PKT_OUT)
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"edge seed {seed}")


def test_edge_corpus_coverage(tables):
    """The corpus must reach (almost) every DoneReason the path can produce."""
    _, tp = tables
    frames = edge_frames(16000, 99)
    buf, inp = pack_burst(frames)
    out = Oracle(tp).process(buf, inp, A.PKT_OUT)
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
