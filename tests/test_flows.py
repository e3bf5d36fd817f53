"""CPU: the flow-table path's known-answer tests (tests/golden/flowkat.py) and
the FlowTable semantics (flow-entry/src/flow_table/table.rs) through the
oracle.  The GPU runs the same cases in tests/test_gpu_flows.py."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from dataplane_amd.flows import NEVER, flow_key, make_flow, reverse_key
from oracle.pyoracle import Oracle, OracleFlows

from golden.flowkat import all_cases, run_case

CASES = all_cases()


class OracleBackend:
    def table(self):
        return OracleFlows()

    def process(self, tb, buf, inp, ft):
        return Oracle(tb.build()).process_flows(buf, inp, ft)


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_flow_kat_oracle(case):
    errs = run_case(case, OracleBackend())
    assert not errs, "\n".join(errs)


def k4(i, vni=100, kind=A.FLOW_UDP):
    return flow_key(vni, f"10.0.{i >> 8}.{i & 255}", "20.0.0.1", kind, 1000 + i, 80)


def table_semantics(ft):
    """FlowTable semantics shared by the oracle and the device table
    (table.rs:134-317, flow_info.rs:290-465); returns nothing, asserts."""
    f0 = make_flow(k4(0), 200, genid=3, expires_at=10)
    refs, res = ft.insert(f0)
    assert res[0] == A.FLOW_INSERTED
    info = ft.lookup(k4(0))[0]
    assert info["ref"] == refs[0] and info["status"] == A.FLOW_ACTIVE
    assert info["dst_vni"] == 200 and info["genid"] == 3 and info["expires_at"] == 10
    assert ft.lookup(k4(1))[0]["ref"] == A.FLOW_NONE
    # the same key again replaces; the old FlowInfo is Detached (out of the table)
    refs2, res2 = ft.insert(make_flow(k4(0), 201))
    assert res2[0] == A.FLOW_REPLACED and refs2[0] != refs[0]
    assert ft.get(refs)[0]["ref"] == A.FLOW_NONE
    assert ft.lookup(k4(0))[0]["dst_vni"] == 201
    assert ft.count() == (1, 1)
    # a port-swapped key is another flow (Hash covers src then dst port)
    swapped = flow_key(100, "10.0.0.0", "20.0.0.1", A.FLOW_UDP, 80, 1000)
    assert ft.lookup(swapped)[0]["ref"] == A.FLOW_NONE
    # capacity: at the limit a new flow is refused
    ft.set_capacity(3)
    _, r = ft.insert(np.array([make_flow(k4(i), 200) for i in (1, 2, 3)], dtype=A.FLOW))
    assert list(r) == [A.FLOW_INSERTED, A.FLOW_INSERTED, A.EFLOWCAP]
    assert ft.count()[0] == 3
    # ... except the second half of a pair whose first half is active
    ft.set_capacity(4)
    a = make_flow(k4(10), 200, A.FLOW_INITIATOR)
    b = make_flow(reverse_key(k4(10), 200), 100)
    pr, pres = ft.insert_pair(a, b)
    assert list(pres) == [A.FLOW_INSERTED, A.FLOW_INSERTED] and ft.count()[0] == 5
    ia, ib = ft.get(pr)
    assert ia["related"] == pr[1] and ib["related"] == pr[0]
    # at the limit with the first half refused, the second is refused too
    pr2, pres2 = ft.insert_pair(make_flow(k4(11), 200, A.FLOW_INITIATOR),
                                make_flow(reverse_key(k4(11), 200), 100))
    assert list(pres2) == [A.EFLOWCAP, A.EFLOWCAP]
    assert list(pr2) == [A.FLOW_NONE, A.FLOW_NONE]
    # invalidate_pair cancels both halves; the timers then remove them
    ft.invalidate([pr[0]])
    ia, ib = ft.get(pr)
    assert ia["status"] == A.FLOW_CANCELLED and ib["status"] == A.FLOW_CANCELLED
    assert ft.count() == (5, 3)
    assert ft.sweep(0) == 2
    assert ft.count() == (3, 3)
    assert ft.get(pr)[0]["ref"] == A.FLOW_NONE
    # expiry: an active flow whose deadline passed is expired and removed;
    # a Detached one stays
    ft.set_capacity(100)
    er, _ = ft.insert(np.array([make_flow(k4(20), 200, expires_at=5),
                                make_flow(k4(21), 200, expires_at=50),
                                make_flow(k4(22), 200, expires_at=5)], dtype=A.FLOW))
    ft.set_status(er[2], A.FLOW_DETACHED)
    assert ft.sweep(5) == 1
    g = ft.get(er)
    assert g[0]["ref"] == A.FLOW_NONE and g[1]["status"] == A.FLOW_ACTIVE
    assert g[2]["status"] == A.FLOW_DETACHED
    # remove
    assert ft.remove(k4(21)) == 1 and ft.remove(k4(21)) == 0
    assert ft.lookup(k4(21))[0]["ref"] == A.FLOW_NONE
    # a removed slot is reusable and lookups probe past it
    r3, _ = ft.insert(make_flow(k4(21), 202))
    assert ft.lookup(k4(21))[0]["dst_vni"] == 202
    # v6 and ICMP keys
    k6 = flow_key(7, "2001:db8::1", "2001:db8::2", A.FLOW_ICMP_QUERY, 0x1234, 0)
    ft.insert(make_flow(k6, 9))
    assert ft.lookup(k6)[0]["dst_vni"] == 9
    ko = flow_key(7, "2001:db8::1", "2001:db8::2", A.FLOW_ICMP_OTHER)
    assert ft.lookup(ko)[0]["ref"] == A.FLOW_NONE


def test_flow_table_semantics_oracle():
    table_semantics(OracleFlows())


def test_flow_insert_rejects_invalid():
    ft = OracleFlows()
    bad = make_flow(k4(0), 0)                      # no destination VPC
    with pytest.raises(RuntimeError):
        ft.insert(bad)
    z = make_flow(flow_key(1, "1.1.1.1", "2.2.2.2", A.FLOW_TCP, 0, 5), 2)  # zero port
    with pytest.raises(RuntimeError):
        ft.insert(z)
    a = make_flow(k4(0), 200)
    with pytest.raises(RuntimeError):              # no initiator
        ft.insert_pair(a, make_flow(reverse_key(k4(0), 200), 100))
    with pytest.raises(RuntimeError):              # identical keys
        ft.insert_pair(make_flow(k4(0), 200, A.FLOW_INITIATOR), a)


def test_burst_request_flows_match_packet_keys():
    """The vectorised flow builder (bench, full-size tests) makes exactly
    FlowKey::try_from of each frame (tests/flowgen.frame_key)."""
    from dataplane_amd.flows import burst_request_flows
    from dataplane_amd.workload import Workload
    from flowgen import frame_key, frames_of
    w = Workload(2, 3000, seed=4, n_routes_v4=1000, n_acl=100, n_nat=8, tcp_percent=30)
    dst = np.full(w.n, 7, np.uint32)
    fl = burst_request_flows(w.buf, w.inp, np.arange(w.n), dst, genid=3)
    want = {frame_key(f, v).tobytes() for f, v in frames_of(w) if v}
    got = {np.ascontiguousarray(k).tobytes() for k in fl["key"]}
    assert got == want and (fl["dst_vni"] == 7).all() and (fl["genid"] == 3).all()
