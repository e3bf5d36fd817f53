"""Known-answer tests of the flow-table path, transcribed
from the reference's own tests of FlowLookup, the flow-aware FlowFilter,
AclFilter and IcmpErrorHandler branches.

The reference tests attach a FlowInfo to a packet by hand; here the flows are
inserted into the flow table and FlowLookup attaches them, then the whole path
runs.  Flows carry no masquerade / port-forwarding state (§8f rank 3), so the
reference tests about that state are restated without it where their
assertions still apply.  The burst-order cases pin the reference's stage order
within one burst (flow-filter/src/lib.rs:75-111: the flow filter runs over the
whole burst before any later stage).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from dataplane_amd import _abi as A
from dataplane_amd.flows import NEVER, flow_key, make_flow, reverse_key
from dataplane_amd.tables import ALLOW, DENY, TablesBuilder
from golden.kat import IF_MAC, NH_MAC, OIF_MAC, icmp4_err_frame, tcp_frame, test_ipv4_frame

TB = TablesBuilder
ACTIVE, CANCELLED, EXPIRED, DETACHED = (A.FLOW_ACTIVE, A.FLOW_CANCELLED, A.FLOW_EXPIRED,
                                        A.FLOW_DETACHED)
GONE = "gone"  # not in the table any more


def vpc_pair_tables(genid: int, ips1: str, ips2: str, acl=(), defaults=(), vni1=100,
                    vni2=200) -> Callable[[], TablesBuilder]:
    """Two peered VPCs, vpc1 exposing ips1 and vpc2 exposing ips2 in both
    directions (no NAT); every VPC routes 0/0 to a resolved next hop.  acl:
    (src_vni, dst_vni, add_acl kwargs); defaults: (src_vni, dst_vni, action)."""
    def build():
        t = TB(genid=genid)
        t.add_iface(1, IF_MAC)
        t.add_iface(10, OIF_MAC)
        t.add_adjacency("192.0.2.1", 10, NH_MAC)
        nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
        t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
        for v in (vni1, vni2, 300):
            t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
        t.add_ff_remote(vni1, ips2, vni2)
        t.add_ff_local(vni1, vni2, ips1)
        t.add_ff_remote(vni2, ips1, vni1)
        t.add_ff_local(vni2, vni1, ips2)
        for (s, d, kw) in acl:
            t.add_acl(s, d, **kw)
        for (s, d, a) in defaults:
            t.add_acl_default(s, d, a)
        return t
    return build


@dataclass
class FPkt:
    frame: bytes
    vni: int                               # seeded source VNI (overlay, post-decap)
    expect: Dict = field(default_factory=dict)   # done / dst_vni / acl / acl_rule / flow


@dataclass
class FCase:
    name: str
    ref: str
    tables: Callable[[], TablesBuilder]
    # flows to insert: (name, dp_flow) or ((name_a, flow_a), (name_b, flow_b)) for a related pair
    flows: List
    packets: List[FPkt]
    status: Dict[str, object] = field(default_factory=dict)   # set before the burst
    sweep_at: Optional[int] = None          # flow timers fired up to this time before the burst
    expect_status: Dict[str, object] = field(default_factory=dict)  # after the burst
    expect_related: Dict[str, Optional[str]] = field(default_factory=dict)


def tcp_key(vni, src, dst, sp, dp):
    return flow_key(vni, src, dst, A.FLOW_TCP, sp, dp)


def pair(key, vni_a, vni_b, genid_a=0, genid_b=None, flags_a=A.FLOW_INITIATOR, flags_b=0,
         exp_a=NEVER, exp_b=NEVER, dst_b=None):
    """FlowInfo::related_pair of `key` (from vni_a towards vni_b) and its
    reverse (from vni_b): create_flow_pair (flow-filter/src/tests.rs:43-79)."""
    a = make_flow(key, vni_b, flags_a, genid_a, exp_a)
    b = make_flow(reverse_key(key, vni_b), vni_a if dst_b is None else dst_b, flags_b,
                  genid_a if genid_b is None else genid_b, exp_b)
    return a, b


def ff_cases() -> List[FCase]:
    ff = "flow-filter/src/tests.rs"
    k = tcp_key(100, "1.0.0.5", "5.0.0.10", 1234, 5678)
    pkt = tcp_frame("1.0.0.5", "5.0.0.10", 1234, 5678)
    t0 = vpc_pair_tables(0, "1.0.0.0/24", "5.0.0.0/24")
    t5 = vpc_pair_tables(5, "1.0.0.0/24", "5.0.0.0/24")
    cs = []
    a, b = pair(k, 100, 200)
    cs.append(FCase("ff_active_flow_is_honored", f"{ff}:403-418 (no masquerade state)", t0,
                    [(("fwd", a), ("rev", b))],
                    [FPkt(pkt, 100, dict(done="Delivered", dst_vni=200, flow="fwd"))],
                    expect_status=dict(fwd=ACTIVE, rev=ACTIVE)))
    a, b = pair(k, 100, 300)
    cs.append(FCase("ff_outdated_flow_is_invalidated", f"{ff}:421-438", t5,
                    [(("fwd", a), ("rev", b))],
                    [FPkt(pkt, 100, dict(done="Delivered", dst_vni=200, flow="fwd"))],
                    expect_status=dict(fwd=CANCELLED, rev=CANCELLED)))
    a, b = pair(k, 100, 200)
    cs.append(FCase("ff_inactive_flow_is_not_honored", f"{ff}:535-550 (no masquerade state)", t0,
                    [(("fwd", a), ("rev", b))],
                    [FPkt(pkt, 100, dict(done="Delivered", dst_vni=200, flow="fwd"))],
                    status=dict(fwd=DETACHED), expect_status=dict(fwd=DETACHED, rev=ACTIVE)))
    a, b = pair(k, 100, 200)
    cs.append(FCase("ff_outdated_flow_no_longer_needing_state_is_invalidated", f"{ff}:570-583",
                    t5, [(("fwd", a), ("rev", b))],
                    [FPkt(pkt, 100, dict(done="Delivered", dst_vni=200, flow="fwd"))],
                    expect_status=dict(fwd=CANCELLED, rev=CANCELLED)))
    k9 = tcp_key(100, "1.0.0.5", "9.9.9.9", 1234, 5678)
    a, b = pair(k9, 100, 200, genid_a=9)
    cs.append(FCase("ff_flow_from_a_newer_generation_is_honored", f"{ff}:2086-2110", t0,
                    [(("fwd", a), ("rev", b))],
                    [FPkt(tcp_frame("1.0.0.5", "9.9.9.9", 1234, 5678), 100,
                          dict(done="Delivered", dst_vni=200, flow="fwd"))],
                    expect_status=dict(fwd=ACTIVE, rev=ACTIVE)))
    a, b = pair(k9, 100, 200, genid_a=0)
    cs.append(FCase("ff_outdated_flow_on_a_miss_is_invalidated",
                    "flow-filter/src/lib.rs:174-185 (apply_route: miss -> invalidate_flows)", t5,
                    [(("fwd", a), ("rev", b))],
                    [FPkt(tcp_frame("1.0.0.5", "9.9.9.9", 1234, 5678), 100,
                          dict(done="Filtered", dst_vni=0, flow="fwd"))],
                    expect_status=dict(fwd=CANCELLED, rev=CANCELLED)))
    return cs


V1, V2 = "10.0.0.0/24", "20.0.0.0/24"


def acl_cases() -> List[FCase]:
    at = "acl-filter/src/tests.rs"
    req = tcp_frame("10.0.0.5", "20.0.0.5", 1234, 80)
    rep = tcp_frame("20.0.0.5", "10.0.0.5", 80, 1234)
    fwd_key = tcp_key(100, "10.0.0.5", "20.0.0.5", 1234, 80)
    allow_flow = (100, 200, dict(action=ALLOW, proto=6, src=V1, dst=V2, scope=A.ACL_SCOPE_FLOW))
    allow_pkt = (100, 200, dict(action=ALLOW, proto=6, src=V1, dst=V2, scope=A.ACL_SCOPE_PACKET))
    deny_rep = (200, 100, dict(action=DENY, proto=6, src=V2, dst=V1, scope=A.ACL_SCOPE_PACKET))
    deny_both = ((100, 200, DENY), (200, 100, DENY))
    allow_both = ((100, 200, ALLOW), (200, 100, ALLOW))
    cs = []
    a, b = pair(fwd_key, 100, 200)
    cs.append(FCase("acl_flow_scope_allows_reply_for_allowed_request", f"{at}:690-721",
                    vpc_pair_tables(0, V1, V2, [allow_flow], deny_both),
                    [(("fwd", a), ("rev", b))],
                    [FPkt(req, 100, dict(done="Delivered", acl=1, acl_rule=0, flow="fwd")),
                     FPkt(rep, 200, dict(done="Delivered", dst_vni=100, acl=6, acl_rule=0,
                                         flow="rev"))],
                    expect_status=dict(fwd=ACTIVE, rev=ACTIVE)))
    cs.append(FCase("acl_packet_scope_denies_reply_for_allowed_request", f"{at}:723-752",
                    vpc_pair_tables(0, V1, V2, [allow_pkt], deny_both),
                    [(("fwd", a), ("rev", b))],
                    [FPkt(req, 100, dict(done="Delivered", acl=1, acl_rule=0, flow="fwd")),
                     FPkt(rep, 200, dict(done="AclDropped", acl=4, flow="rev"))],
                    expect_status=dict(fwd=CANCELLED, rev=CANCELLED)))
    cs.append(FCase("acl_explicit_deny_rule_drops_reply_despite_matching_flow", f"{at}:757-800",
                    vpc_pair_tables(0, V1, V2, [allow_flow, deny_rep], allow_both),
                    [(("fwd", a), ("rev", b))],
                    [FPkt(req, 100, dict(done="Delivered", acl=1, acl_rule=0, flow="fwd")),
                     FPkt(rep, 200, dict(done="AclDropped", acl=2, acl_rule=1, flow="rev"))],
                    expect_status=dict(fwd=CANCELLED, rev=CANCELLED)))
    # a reply with no flow falls to the peering default (acl-filter/src/lib.rs:130-137)
    cs.append(FCase("acl_reply_without_flow_gets_the_default", f"{at}:723-752 (no flow)",
                    vpc_pair_tables(0, V1, V2, [allow_flow], deny_both), [],
                    [FPkt(rep, 200, dict(done="AclDropped", acl=4, flow=None))]))
    # an outdated reply flow is no valid flow for the ACL (lib.rs:86-92); the
    # flow filter, not bypassed, invalidates it as outdated
    a5, b5 = pair(fwd_key, 100, 200, genid_a=0)
    cs.append(FCase("acl_outdated_reply_flow_gets_the_default", "acl-filter/src/lib.rs:71-94",
                    vpc_pair_tables(5, V1, V2, [allow_flow], deny_both),
                    [(("fwd", a5), ("rev", b5))],
                    [FPkt(rep, 200, dict(done="AclDropped", acl=4, flow="rev"))],
                    expect_status=dict(fwd=CANCELLED, rev=CANCELLED)))
    return cs


def lookup_cases() -> List[FCase]:
    lk = "flow-entry/src/flow_table/nf_lookup.rs"
    k = tcp_key(100, "1.2.3.4", "5.6.7.8", 1025, 2048)
    pkt = tcp_frame("1.2.3.4", "5.6.7.8", 1025, 2048)
    t = vpc_pair_tables(0, "1.2.3.0/24", "5.6.7.0/24")
    cs = [FCase("flow_lookup_tags_packet", f"{lk}:83-111", t,
                [("f", make_flow(k, 200))],
                [FPkt(pkt, 100, dict(done="Delivered", dst_vni=200, flow="f")),
                 # a key that differs only in the source VPC is another flow
                 FPkt(pkt, 200, dict(flow=None))],
                expect_status=dict(f=ACTIVE))]
    # test_lookups_with_related_flows: flow_1 expires at 2, flow_2 at 60; after
    # the timers ran up to 3, packet_1 finds no flow and packet_2's flow has
    # lost its related flow
    k1 = flow_key(100, "10.0.0.1", "20.0.0.1", A.FLOW_UDP, 80, 500)
    k2 = flow_key(100, "192.168.1.1", "20.0.0.1", A.FLOW_UDP, 500, 80)
    f1 = make_flow(k1, 200, A.FLOW_INITIATOR, 0, 2)
    f2 = make_flow(k2, 200, 0, 0, 60)
    t2 = vpc_pair_tables(0, "10.0.0.0/8", "20.0.0.0/24")
    from pktgen import udp4_frame
    p1 = udp4_frame(IF_MAC, "02:00:00:00:00:01", "10.0.0.1", "20.0.0.1", 80, 500)
    p2 = udp4_frame(IF_MAC, "02:00:00:00:00:01", "192.168.1.1", "20.0.0.1", 500, 80)
    cs.append(FCase("flow_lookup_related_flows_after_expiry", f"{lk}:182-273", t2,
                    [(("f1", f1), ("f2", f2))],
                    [FPkt(p1, 100, dict(flow=None)), FPkt(p2, 100, dict(flow="f2"))],
                    sweep_at=3, expect_status=dict(f1=GONE, f2=ACTIVE),
                    expect_related=dict(f2=None)))
    cs.append(FCase("flow_lookup_related_flows_before_expiry", f"{lk}:221-242", t2,
                    [(("f1", f1), ("f2", f2))],
                    [FPkt(p1, 100, dict(flow="f1")), FPkt(p2, 100, dict(flow="f2"))],
                    sweep_at=1, expect_status=dict(f1=ACTIVE, f2=ACTIVE),
                    expect_related=dict(f1="f2", f2="f1")))
    return cs


def icmp_cases() -> List[FCase]:
    h = "nat/src/icmp_handler/nf.rs"
    # the embedded (10.2.0.1:1234 -> 10.1.0.1:5678) reversed from VPC 100
    k = tcp_key(100, "10.1.0.1", "10.2.0.1", 5678, 1234)
    err = icmp4_err_frame("10.1.0.1", "10.2.0.1", "10.2.0.1", "10.1.0.1", 6)
    t = vpc_pair_tables(0, "10.1.0.0/24", "10.2.0.0/24")
    return [
        FCase("icmp_error_matching_flow_without_nat_state_is_filtered", f"{h}:102-152", t,
              [("f", make_flow(k, 200))],
              [FPkt(err, 100, dict(done="Filtered", dst_vni=200, flow=None))],
              expect_status=dict(f=ACTIVE)),
        FCase("icmp_error_matching_inactive_flow_is_filtered", f"{h}:124-130", t,
              [("f", make_flow(k, 200))],
              [FPkt(err, 100, dict(done="Filtered", dst_vni=0, flow=None))],
              status=dict(f=CANCELLED), expect_status=dict(f=CANCELLED)),
        FCase("icmp_error_without_matching_flow_passes", f"{h}:113-121", t,
              [("f", make_flow(tcp_key(100, "10.1.0.1", "10.2.0.1", 5679, 1234), 200))],
              [FPkt(err, 100, dict(done="Delivered", dst_vni=200, flow=None))],
              expect_status=dict(f=ACTIVE)),
    ]


def burst_order_cases() -> List[FCase]:
    """One burst, several packets on one flow pair (flow-filter/src/lib.rs:
    75-111, 352-363; nf_lookup.rs / acl-filter/src/lib.rs are lazy per packet)."""
    fwd_key = tcp_key(100, "10.0.0.5", "20.0.0.5", 1234, 80)
    req = tcp_frame("10.0.0.5", "20.0.0.5", 1234, 80)
    rep = tcp_frame("20.0.0.5", "10.0.0.5", 80, 1234)
    allow_flow = (100, 200, dict(action=ALLOW, proto=6, src=V1, dst=V2, scope=A.ACL_SCOPE_FLOW))
    deny_both = ((100, 200, DENY), (200, 100, DENY))
    t5 = vpc_pair_tables(5, V1, V2, [allow_flow], deny_both)
    # the request's flow is outdated (genid 0 < 5), the reply's current (5)
    a, b = pair(fwd_key, 100, 200, genid_a=0, genid_b=5)
    why = "flow-filter/src/lib.rs:75-111,258-294; acl-filter/src/lib.rs:71-128"
    return [
        FCase("burst_reply_alone_allowed_by_its_flow", why, t5, [(("fwd", a), ("rev", b))],
              [FPkt(rep, 200, dict(done="Delivered", acl=6, flow="rev"))],
              expect_status=dict(fwd=ACTIVE, rev=ACTIVE)),
        # the request, later in the burst, invalidates the pair in the flow
        # filter, which runs before the reply's ACL
        FCase("burst_flow_filter_invalidation_precedes_every_acl", why, t5,
              [(("fwd", a), ("rev", b))],
              [FPkt(rep, 200, dict(done="AclDropped", acl=4, flow="rev")),
               FPkt(req, 100, dict(done="Delivered", acl=1, flow="fwd"))],
              expect_status=dict(fwd=CANCELLED, rev=CANCELLED)),
        FCase("burst_flow_filter_invalidation_request_first", why, t5,
              [(("fwd", a), ("rev", b))],
              [FPkt(req, 100, dict(done="Delivered", acl=1, flow="fwd")),
               FPkt(rep, 200, dict(done="AclDropped", acl=4, flow="rev")),
               FPkt(rep, 200, dict(done="AclDropped", acl=4, flow="rev"))],
              expect_status=dict(fwd=CANCELLED, rev=CANCELLED)),
    ]


def all_cases() -> List[FCase]:
    return ff_cases() + acl_cases() + lookup_cases() + icmp_cases() + burst_order_cases()


# ------------------------------------------------------------------ runner

def run_case(case: FCase, backend) -> List[str]:
    """backend: .table() -> a flow table (FlowTable / OracleFlows);
    .process(tables_builder, buf, inp, table) -> (out, flow_refs)."""
    from edgecase import pack_burst
    ft = backend.table()
    refs: Dict[str, int] = {}
    for item in case.flows:
        if isinstance(item[0], tuple):
            (na, fa), (nb, fb) = item
            r, res = ft.insert_pair(fa, fb)
            refs[na], refs[nb] = int(r[0]), int(r[1])
        else:
            n, f = item
            r, res = ft.insert(f)
            refs[n] = int(r[0])
    for n, st in case.status.items():
        ft.set_status(refs[n], st)
    if case.sweep_at is not None:
        ft.sweep(case.sweep_at)
    name_of = {v: k for k, v in refs.items()}
    frames = [(p.frame, 1, A.IN_SEEDED_OVERLAY, p.vni) for p in case.packets]
    buf, inp = pack_burst(frames)
    out, frefs = backend.process(case.tables(), buf, inp, ft)
    errs = []
    for i, p in enumerate(case.packets):
        o, e = out[i], p.expect
        tag = f"{case.name}[{i}] ({case.ref})"
        done = A.DONE_NAMES[o["done"]] if o["done"] < A.DONE_COUNT else int(o["done"])
        if "done" in e and done != e["done"]:
            errs.append(f"{tag}: done {done} != {e['done']}")
        for k in ("dst_vni", "acl"):
            if k in e and int(o[k]) != e[k]:
                errs.append(f"{tag}: {k} {int(o[k])} != {e[k]}")
        if "acl_rule" in e:
            got = None if o["acl_rule"] == 0xFFFFFFFF else int(o["acl_rule"])
            if got != e["acl_rule"]:
                errs.append(f"{tag}: acl_rule {got} != {e['acl_rule']}")
        if "flow" in e:
            got = None if int(frefs[i]) == A.FLOW_NONE else name_of.get(int(frefs[i]), "?")
            if got != e["flow"]:
                errs.append(f"{tag}: flow {got} != {e['flow']}")
    if case.expect_status or case.expect_related:
        names = sorted(refs)
        info = ft.get([refs[n] for n in names])
        for n, inf in zip(names, info):
            gone = int(inf["ref"]) == A.FLOW_NONE
            if n in case.expect_status:
                want = case.expect_status[n]
                got = GONE if gone else int(inf["status"])
                if got != want:
                    errs.append(f"{case.name}: flow {n} status {got} != {want}")
            if n in case.expect_related and not gone:
                rel = None if int(inf["related"]) == A.FLOW_NONE else name_of.get(int(inf["related"]))
                if rel != case.expect_related[n]:
                    errs.append(f"{case.name}: flow {n} related {rel} != {case.expect_related[n]}")
    return errs
