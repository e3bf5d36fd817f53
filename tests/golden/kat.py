"""Known-answer tests transcribed from the reference's own tests.

Each case builds tables (dataplane_amd.tables.TablesBuilder) and frames
(tests/pktgen.py), runs them through the whole path, and checks the values the
cited reference test asserts.  The expected values are the reference's; they
pin the oracle and the HIP path alike (SURVEY.md §8c "Golden vectors and KATs").

Observation model: the reference tests call one stage; here the whole path
runs, so surrounding stages are configured to be transparent (wildcard
flow-filter rules, a 0/0 egress route) and only the fields the reference test
asserts are checked.
"""
from __future__ import annotations

import ipaddress
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from dataplane_amd import _abi as A
from dataplane_amd.tables import (ALLOW, DENY, NAT_NONE, NAT_STATIC, TablesBuilder)
import pktgen as P
from golden import natcfg as N

TB = TablesBuilder
IF_MAC = "02:00:00:00:00:02"      # build_test_ipv4_packet dst MAC (net/src/packet/test_utils.rs:65-71)
PEER_MAC = "02:00:00:00:00:01"    # ... and its src MAC
OIF_MAC = "02:00:00:00:00:10"
NH_MAC = "02:00:00:00:77:01"


@dataclass
class Pkt:
    frame: bytes
    iif: int = 1
    seeded_vni: int = 0            # DP_IN_SEEDED_OVERLAY with this src VNI when != 0
    expect: Dict = field(default_factory=dict)


@dataclass
class Case:
    name: str
    ref: str                       # reference test file:line
    tables: Callable[[], TablesBuilder]
    packets: List[Pkt]
    passes: int = 1                # re-inject delivered frames this many times


# ---------------------------------------------------------------- frames

def test_ipv4_frame(src="1.2.3.4", dst="5.6.7.8", ttl=255, proto=None, sport=123, dport=456,
                    dscp=0, ecn=0, dmac=IF_MAC, smac=PEER_MAC) -> bytes:
    """build_test_ipv4_packet(_with_transport) (net/src/packet/test_utils.rs:85-127):
    Eth 02:..:01 -> 02:..:02, IPv4 1.2.3.4 -> 5.6.7.8, ports 123 -> 456."""
    if proto is None:
        ip = P.ipv4(src, dst, 255, 0, ttl=ttl, dscp=dscp, ecn=ecn)
        return P.eth(dmac, smac, 0x0800) + ip
    body = P.l4(proto, sport, dport, b"", P.pseudo4(src, dst, proto, 8 if proto == 17 else 20))
    return P.eth(dmac, smac, 0x0800) + P.ipv4(src, dst, proto, len(body), ttl=ttl, dscp=dscp,
                                              ecn=ecn) + body


def tcp_frame(src, dst, sport, dport, **kw):
    return test_ipv4_frame(src, dst, proto=6, sport=sport, dport=dport, **kw)


# ---------------------------------------------------------------- tables

def overlay_tables(src_vni=100, dst_vni=200, acl=None, acl_default=None, ff_remote=None,
                   nat=None, nat_flags=(NAT_NONE, NAT_NONE), extra_vnis=()) -> TablesBuilder:
    """Two VPCs; every flow-filter rule wildcard unless given; dst VPC routes
    0/0 to a resolved next hop on oif 10."""
    t = TB()
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    und = t.add_fib(0)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(und, "0.0.0.0/0", nh)
    for v in sorted({src_vni, dst_vni, *extra_vnis}):
        f = t.add_fib(v, vnis=[v])
        t.add_route(f, "0.0.0.0/0", nh)
        t.add_route(f, "::/0", nh)
    if ff_remote is None:
        t.add_ff_remote(src_vni, "0.0.0.0/0", dst_vni, nat_flags[1])
        t.add_ff_remote(src_vni, "::/0", dst_vni)
    else:
        for (pfx, vni) in ff_remote:
            t.add_ff_remote(src_vni, pfx, vni)
    for v in sorted({dst_vni, *extra_vnis}):
        t.add_ff_local(src_vni, v, "0.0.0.0/0", nat_flags[0])
        t.add_ff_local(src_vni, v, "::/0")
    for r in acl or []:
        t.add_acl(src_vni, dst_vni, **r)
    if acl_default is not None:
        t.add_acl_default(src_vni, dst_vni, acl_default)
    if nat is not None:
        N.lower(t, nat)
    return t


DROP_10_8_TO_22 = dict(action=DENY, proto=6, src="10.0.0.0/8", dports=(22, 22))
ALLOW_ALL_TCP = dict(action=ALLOW, proto=6)


def acl_cases() -> List[Case]:
    ov = tcp_frame("10.1.2.3", "192.168.1.1", 54321, 22)
    cs = [
        Case("acl_single_rule_hit_and_miss", "acl/src/reference/table.rs:144-178",
             lambda: overlay_tables(acl=[DROP_10_8_TO_22]), [
                 Pkt(ov, seeded_vni=100, expect=dict(done="AclDropped", acl=2, acl_rule=0)),
                 Pkt(tcp_frame("11.0.0.1", "192.168.1.1", 54321, 22), seeded_vni=100,
                     expect=dict(done="Delivered", acl=5)),
                 Pkt(tcp_frame("10.1.2.3", "192.168.1.1", 54321, 80), seeded_vni=100,
                     expect=dict(done="Delivered", acl=5)),
             ]),
        Case("acl_empty_table_always_misses", "acl/src/reference/table.rs:180-194",
             lambda: overlay_tables(acl=[]), [
                 Pkt(tcp_frame("0.0.0.0", "0.0.0.0", 0, 0), seeded_vni=100,
                     expect=dict(done="Delivered", acl=5, acl_rule=None)),
             ]),
        Case("acl_positional_precedence_first_match_wins", "acl/src/reference/table.rs:221-225",
             lambda: overlay_tables(acl=[ALLOW_ALL_TCP, DROP_10_8_TO_22]), [
                 Pkt(ov, seeded_vni=100, expect=dict(done="Delivered", acl=1, acl_rule=0)),
             ]),
        Case("acl_later_rule_after_miss", "acl-filter/src/fuzz.rs:229-270",
             lambda: overlay_tables(acl=[dict(action=ALLOW, proto=17), DROP_10_8_TO_22]), [
                 Pkt(ov, seeded_vni=100, expect=dict(done="AclDropped", acl=2, acl_rule=1)),
             ]),
        Case("acl_default_action_for_peering", "acl-filter/src/context.rs:564-566",
             lambda: overlay_tables(acl=[DROP_10_8_TO_22], acl_default=DENY), [
                 Pkt(tcp_frame("11.0.0.1", "192.168.1.1", 54321, 22), seeded_vni=100,
                     expect=dict(done="AclDropped", acl=4)),
                 Pkt(ov, seeded_vni=100, expect=dict(done="AclDropped", acl=2, acl_rule=0)),
             ]),
        Case("acl_absent_default_allows", "acl-filter/src/fuzz.rs:319-340",
             lambda: overlay_tables(acl=[DROP_10_8_TO_22]), [
                 Pkt(tcp_frame("11.0.0.1", "192.168.1.1", 1, 2), seeded_vni=100,
                     expect=dict(done="Delivered", acl=5)),
             ]),
    ]
    # prefix masks /24 /20 /0 /32 (match-action/src/predicate.rs:283-288)
    masks = [dict(action=DENY, dst="10.1.2.0/24"), dict(action=DENY, dst="172.16.0.0/20"),
             dict(action=DENY, dst="192.0.2.7/32"), dict(action=DENY, proto=17, dports=(9999, 9999))]
    u = lambda dst, dport=53: test_ipv4_frame("10.9.9.9", dst, proto=17, dport=dport)  # noqa: E731
    cs.append(Case("prefix_mask_sets_top_bits", "match-action/src/predicate.rs:283-288",
                   lambda: overlay_tables(acl=masks), [
                       Pkt(u("10.1.2.255"), seeded_vni=100, expect=dict(done="AclDropped", acl_rule=0)),
                       Pkt(u("10.1.3.0"), seeded_vni=100, expect=dict(done="Delivered")),
                       Pkt(u("172.16.15.255"), seeded_vni=100, expect=dict(done="AclDropped", acl_rule=1)),
                       Pkt(u("172.16.16.0"), seeded_vni=100, expect=dict(done="Delivered")),
                       Pkt(u("192.0.2.7"), seeded_vni=100, expect=dict(done="AclDropped", acl_rule=2)),
                       Pkt(u("192.0.2.8"), seeded_vni=100, expect=dict(done="Delivered")),
                       Pkt(u("203.0.113.1", 9999), seeded_vni=100, expect=dict(done="AclDropped", acl_rule=3)),
                   ]))
    return cs


def ff_cases() -> List[Case]:
    # rule_priority is lexicographic in (prefix length, port forwarding)
    # (flow-filter/src/context/tables.rs:452-454, test :969-995): the longer
    # prefix wins whatever the insertion order.
    def tabs(order):
        rules = [("10.0.0.0/8", 300), ("10.1.0.0/16", 200)]
        return overlay_tables(ff_remote=rules if order else rules[::-1], extra_vnis=(300,))
    out = []
    for order in (0, 1):
        out.append(Case(f"ff_priority_longer_prefix_wins_{order}",
                        "flow-filter/src/context/tables.rs:969-995",
                        lambda o=order: tabs(o), [
                            Pkt(test_ipv4_frame("1.1.1.1", "10.1.2.3"), seeded_vni=100,
                                expect=dict(done="Delivered", dst_vni=200)),
                            Pkt(test_ipv4_frame("1.1.1.1", "10.2.0.1"), seeded_vni=100,
                                expect=dict(done="Delivered", dst_vni=300)),
                            Pkt(test_ipv4_frame("1.1.1.1", "11.0.0.1"), seeded_vni=100,
                                expect=dict(done="Filtered")),
                        ]))
    return out


def lpm_cases() -> List[Case]:
    """routing/src/rib/vrf.rs:893-935: /32 routes resolve to themselves (two
    next hops each); once deleted, lookups resolve to the default drop that
    Fib::default installs for v4 and v6 (routing/src/fib/fibtype.rs:76-91)."""
    def tabs(with_routes: bool):
        t = TB()
        t.add_iface(1, IF_MAC)
        t.add_iface(2, "02:00:00:00:00:12")
        t.add_iface(3, "02:00:00:00:00:13")
        t.add_adjacency("10.0.0.1", 2, "02:00:00:00:99:01")
        t.add_adjacency("10.0.0.2", 3, "02:00:00:00:99:02")
        f = t.add_fib(0)           # no explicit /0: the compiler installs the drop default
        if with_routes:
            nh = t.add_nh([[TB.egress(2, "10.0.0.1")], [TB.egress(3, "10.0.0.2")]])
            for i in range(1, 11):
                t.add_route(f, f"7.0.0.{i}/32", nh)
        return t
    pk = [Pkt(test_ipv4_frame("1.1.1.1", f"7.0.0.{i}", ttl=64),
              expect=dict(done="Delivered", oif_in=(2, 3), fib_entry_in=(0, 1))) for i in range(1, 11)]
    pk.append(Pkt(test_ipv4_frame("1.1.1.1", "7.0.0.11", ttl=64), expect=dict(done="RouteDrop")))
    v6 = P.eth(IF_MAC, PEER_MAC, 0x86dd) + P.ipv6("2001:db8::1", "2001:db8::2", 59, 0)
    pk.append(Pkt(v6, expect=dict(done="RouteDrop")))
    deleted = [Pkt(test_ipv4_frame("1.1.1.1", f"7.0.0.{i}", ttl=64), expect=dict(done="RouteDrop"))
               for i in range(1, 11)]
    return [Case("lpm_slash32_resolves_to_itself", "routing/src/rib/vrf.rs:893-920",
                 lambda: tabs(True), pk),
            Case("lpm_deleted_resolves_to_default_drop", "routing/src/rib/vrf.rs:921-935",
                 lambda: tabs(False), deleted)]


def ttl_cases() -> List[Case]:
    """pipeline/src/lib.rs:133-164: 150 TTL decrements from 255 leave 105.
    Here: 150 passes through the router (IP-Forward decrements once per
    pass); the adjacency MAC equals the ingress MAC so each delivered frame
    is accepted again."""
    def tabs():
        t = TB()
        t.add_iface(1, IF_MAC)
        t.add_adjacency("192.0.2.1", 1, IF_MAC)
        f = t.add_fib(0)
        t.add_route(f, "0.0.0.0/0", t.add_nh([[TB.egress(1, "192.0.2.1")]]))
        return t
    return [Case("ttl_150_decrements", "pipeline/src/lib.rs:133-164", tabs,
                 [Pkt(test_ipv4_frame(ttl=255), expect=dict(done="Delivered", ttl=105))],
                 passes=150)]


def vxlan_qos_cases() -> List[Case]:
    """net/src/packet/mod.rs:847-889: decap then encap keeps the outer DSCP 46
    and ECN 3, for an IPv4 and an IPv6 underlay."""
    def tabs(v6: bool):
        t = TB()
        t.add_iface(1, IF_MAC)
        t.add_iface(10, OIF_MAC)
        t.add_adjacency("192.0.2.1", 10, NH_MAC)
        vtep, remote = ("2001:db8::1", "2001:db8::2") if v6 else ("10.0.0.1", "10.0.0.2")
        und = t.add_fib(0, vtep_ip=vtep, vtep_mac=IF_MAC)
        t.add_route(und, vtep + ("/128" if v6 else "/32"), t.add_nh([[TB.local(1)]]))
        src = t.add_fib(100, vtep_ip=vtep, vtep_mac=IF_MAC, vnis=[100])
        dst = t.add_fib(200, vtep_ip=vtep, vtep_mac=IF_MAC, vnis=[200])
        nh = t.add_nh([[TB.encap(200, remote, "02:00:00:00:88:01"), TB.egress(10, "192.0.2.1")]])
        t.add_route(dst, "0.0.0.0/0", nh)
        t.add_route(src, "0.0.0.0/0", nh)
        t.add_ff_remote(100, "0.0.0.0/0", 200)
        t.add_ff_local(100, 200, "0.0.0.0/0")
        return t

    def frame(v6: bool):
        inner = test_ipv4_frame("1.2.3.4", "5.6.7.8", ttl=64, proto=17, dmac="02:00:00:00:aa:01",
                                smac="02:00:00:00:bb:01")
        vx = P.vxlan(100)
        if v6:
            u = P.udp(50000, 4789, vx + inner, P.pseudo6("2001:db8::2", "2001:db8::1", 17,
                                                        8 + len(vx) + len(inner)))
            ip = P.ipv6("2001:db8::2", "2001:db8::1", 17, len(u), tc=(46 << 2) | 3)
            return P.eth(IF_MAC, PEER_MAC, 0x86dd) + ip + u
        u = P.udp(50000, 4789, vx + inner, csum=0)
        ip = P.ipv4("10.0.0.2", "10.0.0.1", 17, len(u), dscp=46, ecn=3)
        return P.eth(IF_MAC, PEER_MAC, 0x0800) + ip + u
    return [Case(f"vxlan_decap_encap_keeps_outer_qos_{'v6' if v6 else 'v4'}",
                 "net/src/packet/mod.rs:847-889", lambda v=v6: tabs(v),
                 [Pkt(frame(v6), expect=dict(done="Delivered", outer_dscp=46, outer_ecn=3,
                                             dst_vni=200))])
            for v6 in (False, True)]


def parse_cases() -> List[Case]:
    """dataplane/src/drivers/kernel/worker.rs:650-692: a good frame parses,
    four 0xff bytes do not (the driver drops it: parse error)."""
    def tabs():
        t = TB()
        t.add_iface(1, IF_MAC)
        t.add_iface(10, OIF_MAC)
        t.add_adjacency("192.0.2.1", 10, NH_MAC)
        f = t.add_fib(0)
        t.add_route(f, "0.0.0.0/0", t.add_nh([[TB.egress(10, "192.0.2.1")]]))
        return t
    return [Case("parse_good_and_unparseable", "dataplane/src/drivers/kernel/worker.rs:650-692",
                 tabs, [Pkt(test_ipv4_frame(ttl=64), expect=dict(done="Delivered", ttl=63)),
                        Pkt(b"\xff" * 4, expect=dict(done="NotEthernet"))])]


# ------------------------------------------------------------------ NAT

def dst_nat_static_44_config():
    """build_context (nat/src/static_nat/test.rs:121-274)."""
    e1 = N.Expose(ips=["1.1.0.0/16", "1.2.0.0/16"],
                  nots=["1.1.5.0/24", "1.1.3.0/24", "1.1.1.0/24", "1.2.2.0/24"],
                  as_range=["2.2.0.0/16", "2.1.0.0/16"],
                  not_as=["2.1.8.0/24", "2.2.10.0/24", "2.2.1.0/24", "2.2.2.0/24"])
    e2 = N.Expose(ips=["3.0.0.0/16"], as_range=["4.0.0.0/16"])
    e3 = N.Expose(ips=["8.0.0.0/17", "9.0.0.0/17"], nots=["8.0.0.0/24"],
                  as_range=["3.0.0.0/16"], not_as=["3.0.1.0/24"])
    e4 = N.Expose(ips=["10.0.0.0/16"], nots=["10.0.1.0/24", "10.0.2.0/24"],
                  as_range=["5.5.0.0/17", "5.6.0.0/17"], not_as=["5.6.0.0/24", "5.6.8.0/24"])
    m1, m2 = [e1, e2], [e3, e4]
    return N.nat_tables([N.Peering(100, 200, m1, m2), N.Peering(200, 100, m2, m1)])


def full_config():
    """build_sample_config (nat/src/static_nat/test.rs:379-560)."""
    E = N.Expose
    e121 = E(["1.1.0.0/16"], as_range=["10.12.0.0/16"])
    e122 = E(["1.2.0.0/16"], as_range=["10.98.128.0/17", "10.99.0.0/17"])
    e123 = E(["1.3.0.0/24"], as_range=["10.100.0.0/24"])
    e211 = E(["1.2.2.0/24"], as_range=["10.201.201.0/24"])
    e212 = E(["1.2.3.0/24"], as_range=["10.201.202.0/24"])
    e213 = E(["2.0.0.0/24"], as_range=["10.201.203.0/24"])
    e214 = E(["2.0.1.0/28"], as_range=["10.201.204.192/28"])
    e131 = E(["1.1.0.0/16"], as_range=["3.3.0.0/16"])
    e132 = E(["1.2.0.0/16"], as_range=["3.1.0.0/16", "3.2.0.0/17"], not_as=["3.1.128.0/17"])
    e311 = E(["192.168.128.0/24"], as_range=["3.3.3.0/24"])
    e141 = E(["1.1.0.0/16"], as_range=["4.4.0.0/16"])
    e411 = E(["1.1.0.0/16"], as_range=["4.5.0.0/16"])
    e241 = E(["2.4.0.0/16"], nots=["2.4.1.0/24"], as_range=["44.0.0.0/16"],
             not_as=["44.0.200.0/24"])
    e421 = E(["4.4.0.0/16"], nots=["4.4.128.0/18"], as_range=["44.4.0.0/16"],
             not_as=["44.4.64.0/18"])
    e341 = E(["192.168.100.0/24"], as_range=["34.34.34.0/24"])
    e431 = E(["4.4.0.0/24"], nat=False)
    m12, m21 = [e121, e122, e123], [e211, e212, e213, e214]
    m13, m31 = [e131, e132], [e311]
    m14, m41 = [e141], [e411]
    m24, m42 = [e241], [e421]
    m34, m43 = [e341], [e431]
    pe = []
    for (a, b, ma, mb) in [(100, 200, m12, m21), (300, 100, m31, m13), (100, 400, m14, m41),
                           (200, 400, m24, m42), (300, 400, m34, m43)]:
        pe += [N.Peering(a, b, ma, mb), N.Peering(b, a, mb, ma)]
    return N.nat_tables(pe)


def nat_case(name, ref, cfg, s, d, src, dst, want_src, want_dst):
    return Case(name, ref,
                lambda: overlay_tables(src_vni=s, dst_vni=d, nat=cfg(),
                                       nat_flags=(NAT_STATIC, NAT_STATIC)),
                [Pkt(test_ipv4_frame(src, dst, ttl=255), seeded_vni=s,
                     expect=dict(done="Delivered", src=want_src, dst=want_dst))])


def nat_cases() -> List[Case]:
    cs = [
        nat_case("nat_dst_static_44", "nat/src/static_nat/test.rs:276-331",
                 dst_nat_static_44_config, 100, 200, "1.2.3.4", "5.6.7.8", "2.2.0.4", "10.0.136.8"),
        nat_case("nat_dst_static_44_reply", "nat/src/static_nat/test.rs:276-331",
                 dst_nat_static_44_config, 200, 100, "10.0.136.8", "2.2.0.4", "5.6.7.8", "1.2.3.4"),
    ]
    ref = "nat/src/static_nat/test.rs:630-786"
    vec = [  # (src_vni, dst_vni, orig src, orig dst, target src, target dst)
        (100, 200, "8.8.8.8", "9.9.9.9", "8.8.8.8", "9.9.9.9"),
        (100, 200, "1.1.2.3", "10.201.201.18", "10.12.2.3", "1.2.2.18"),
        (100, 200, "1.2.129.3", "10.201.201.22", "10.99.1.3", "1.2.2.22"),
        (100, 200, "1.3.0.7", "10.201.204.193", "10.100.0.7", "2.0.1.1"),
        (100, 300, "1.1.3.3", "3.3.3.3", "3.3.3.3", "192.168.128.3"),
        (100, 300, "1.2.130.1", "3.3.3.3", "3.2.2.1", "192.168.128.3"),
        (100, 400, "1.1.1.1", "4.5.1.1", "4.4.1.1", "1.1.1.1"),
        (200, 400, "2.4.255.255", "44.4.0.0", "44.0.255.255", "4.4.0.0"),
        (200, 400, "2.4.2.1", "44.4.136.2", "44.0.1.1", "4.4.72.2"),
        (300, 400, "192.168.100.34", "4.4.0.43", "34.34.34.34", "4.4.0.43"),
    ]
    for k, (s, d, a, b, ta, tb) in enumerate(vec):
        cs.append(nat_case(f"nat_full_config_{k}", ref, full_config, s, d, a, b, ta, tb))
        if k:  # reverse path
            cs.append(nat_case(f"nat_full_config_{k}_reverse", ref, full_config, d, s, tb, ta, b, a))
    return cs


def pat_case(name, ref, cfg, s, d, src, sport, dst, dport, want):
    """check_packet_with_ports (nat/src/static_nat/test.rs:820-848): a TCP
    packet, both static-NAT requirements set; `want` = (src, sport, dst, dport)."""
    ws, wsp, wd, wdp = want
    return Case(name, ref,
                lambda: overlay_tables(src_vni=s, dst_vni=d, nat=cfg(),
                                       nat_flags=(NAT_STATIC, NAT_STATIC)),
                [Pkt(tcp_frame(src, dst, sport, dport, ttl=255), seeded_vni=s,
                     expect=dict(done="Delivered", src=ws, dst=wd, sport=wsp, dport=wdp))])


def pat_peering(left: List[N.Expose], right: List[N.Expose]):
    """build_gwconfig_from_exposes (test.rs:787-818): VPC-1 (VNI 100) and
    VPC-2 (VNI 200) peered with the given exposes."""
    return N.nat_tables([N.Peering(100, 200, left, right), N.Peering(200, 100, right, left)])


def pat_basic_config():
    """test_config_with_port_ranges_basic (test.rs:850-869)."""
    e1 = N.Expose(ips=[("1.1.0.0/16", (4001, 5000))], as_range=[("10.1.0.0/16", (8001, 9000))])
    e2 = N.Expose(ips=[("10.2.0.0/16", (1, 5))], nat=False)
    return pat_peering([e1], [e2])


def pat_complex_config():
    """test_config_with_port_ranges_complex (test.rs:914-990)."""
    e1 = N.Expose(ips=[("1.1.1.0/24", (4001, 5000)), ("1.1.2.0/25", (4001, 5000)),
                       ("1.1.3.0/25", (5001, 5500))],
                  nots=[("1.1.1.64/26", (4001, 5000)), ("1.1.1.128/25", (4501, 5000))],
                  as_range=[("10.1.0.0/30", (2001, 2300)), ("10.1.0.128/25", (2001, 3000)),
                            ("10.1.1.0/25", (2501, 3000)), ("10.1.1.128/25", (3001, 4000)),
                            ("10.1.2.3/32", (1, 37200))],
                  not_as=[("10.1.1.128/25", (3456, 3755))])
    e2 = N.Expose(ips=[("2.1.0.0/32", (1, 32768)), ("2.1.0.1/32", (1, 32768))],
                  as_range=[("10.2.0.0/30", (1, 16384))])
    return pat_peering([e1], [e2])


def pat_default_config():
    """test_config_with_port_ranges_with_default (test.rs:1152-1180); the
    default expose (`set_default`) carries no NAT."""
    e1 = N.Expose(ips=[("1.1.0.0/16", (4001, 5000))], as_range=[("10.1.0.0/16", (8001, 9000))])
    e2 = N.Expose(ips=[("1.2.0.0/16", (2001, 3000))], as_range=[("10.2.0.0/16", (6001, 7000))])
    e3 = N.Expose(ips=[], nat=False)
    return pat_peering([e1], [e2, e3])


def pat_doc_example_config():
    """The worked example of PortAddrTranslationValue's doc comment
    (nat/src/static_nat/setup/tables.rs:357-382): 1.0.0.0/24 ports
    4001-5000 onto 2.0.0.0/25 ports 6001-7000 then 3.0.0.0/26 ports
    8001-10000."""
    e1 = N.Expose(ips=[("1.0.0.0/24", (4001, 5000))],
                  as_range=[("2.0.0.0/25", (6001, 7000)), ("3.0.0.0/26", (8001, 10000))])
    return pat_peering([e1], [N.Expose(ips=["9.0.0.0/8"], nat=False)])


def pat_cases() -> List[Case]:
    cs = []
    vec = [  # (config, ref, forward (src, sport, dst, dport), expected translation)
        (pat_basic_config, "nat/src/static_nat/test.rs:875-908",
         ("1.1.2.3", 4024, "10.2.2.18", 1), ("10.1.2.3", 8024, "10.2.2.18", 1)),
        (pat_complex_config, "nat/src/static_nat/test.rs:999-1033",
         ("1.1.1.0", 4001, "10.2.0.0", 1), ("10.1.0.0", 2001, "2.1.0.0", 1)),
        (pat_complex_config, "nat/src/static_nat/test.rs:1037-1071",
         ("1.1.3.127", 5500, "10.2.0.3", 16384), ("10.1.2.3", 37200, "2.1.0.1", 32768)),
        (pat_complex_config, "nat/src/static_nat/test.rs:1075-1109",
         ("1.1.1.255", 4500, "10.2.0.1", 16384), ("10.1.0.254", 2800, "2.1.0.0", 32768)),
        (pat_complex_config, "nat/src/static_nat/test.rs:1113-1147",
         ("1.1.2.0", 4001, "10.2.0.2", 1), ("10.1.0.254", 2801, "2.1.0.1", 1)),
        (pat_default_config, "nat/src/static_nat/test.rs:1184-1219",
         ("1.1.2.3", 4024, "10.2.2.18", 7000), ("10.1.2.3", 8024, "1.2.2.18", 3000)),
        (pat_default_config, "nat/src/static_nat/test.rs:1221-1255",
         ("1.1.2.3", 4024, "123.123.123.123", 7000), ("10.1.2.3", 8024, "123.123.123.123", 7000)),
        # the doc comment's (IP 3.0.0.7) answer; its "port 3" is the offset into
        # 8001-10000, i.e. port 8003
        (pat_doc_example_config, "nat/src/static_nat/setup/tables.rs:357-382",
         ("1.0.0.142", 4003, "9.1.2.3", 80), ("3.0.0.7", 8003, "9.1.2.3", 80)),
    ]
    for k, (cfg, ref, (a, ap, b, bp), want) in enumerate(vec):
        cs.append(pat_case(f"pat_{cfg.__name__}_{k}", ref, cfg, 100, 200, a, ap, b, bp, want))
        if cfg is not pat_doc_example_config:   # reverse path restores the original
            ws, wsp, wd, wdp = want
            cs.append(pat_case(f"pat_{cfg.__name__}_{k}_reverse", ref, cfg, 200, 100, wd, wdp, ws,
                               wsp, (b, bp, a, ap)))
    return cs


# ------------------------------------------------------- ICMP error messages

def icmp4_err_frame(osrc, odst, isrc, idst, inner_proto=6, p1=1234, p2=5678, typ=3, code=0,
                    rest=b"\0\0\0\0", bad_icmp_ck=False, inner=True, inner_ttl=4, ttl=8):
    """build_test_icmp4_destination_unreachable_packet (net/src/packet/
    test_utils.rs:314-400): Eth / IPv4 (ttl 8) / ICMP Destination Unreachable
    (Network) / embedded IPv4 (ttl 4) / full TCP, UDP or ICMP echo header;
    every checksum valid unless asked otherwise."""
    if not inner:
        emb = b""
    else:
        if inner_proto == 6:
            t = P.tcp(p1, p2, b"", P.pseudo4(isrc, idst, 6, 20))
        elif inner_proto == 17:
            t = P.udp(p1, p2, b"", P.pseudo4(isrc, idst, 17, 8))
        elif inner_proto == 1:
            t = P.icmp4(8, 0, struct.pack("!HH", p1, p2))
        elif inner_proto == -1:          # an ICMP error inside: no identifier
            t, inner_proto = P.icmp4(3, 1, b"\0\0\0\0"), 1
        else:                            # a protocol with no embedded transport parser
            t = b""
        emb = P.ipv4(isrc, idst, inner_proto, len(t), ttl=inner_ttl) + t
    body = P.icmp4(typ, code, rest, emb)
    if bad_icmp_ck:
        body = body[:2] + bytes([body[2] ^ 0xFF]) + body[3:]
    return P.eth(IF_MAC, PEER_MAC, 0x0800) + P.ipv4(osrc, odst, 1, len(body), ttl=ttl) + body


def icmp_error_cases() -> List[Case]:
    """ICMP error messages: the IcmpErrorHandler with an empty flow table
    (nat/src/icmp_handler/nf.rs:61-120), static NAT of the embedded packet
    (nat/src/static_nat/nf.rs:111-155) and the checksum refresh at serialize
    (net/src/headers/mod.rs:894-928)."""
    ov = lambda **kw: overlay_tables(**kw)  # noqa: E731
    h = "nat/src/icmp_handler/nf.rs"
    return [
        # test_nat_icmp_error_msg_static_44: (10.0.0.1 -> 2.1.0.1) back to
        # (5.5.0.1 -> 1.1.0.1), its embedded (2.1.0.1 -> 10.0.0.1) back to
        # (1.1.0.1 -> 5.5.0.1)
        Case("icmp_error_static_nat_44", "nat/src/static_nat/test.rs:333-374",
             lambda: overlay_tables(src_vni=200, dst_vni=100, nat=dst_nat_static_44_config(),
                                    nat_flags=(NAT_STATIC, NAT_STATIC)),
             [Pkt(icmp4_err_frame("10.0.0.1", "2.1.0.1", "2.1.0.1", "10.0.0.1"), seeded_vni=200,
                  expect=dict(done="Delivered", src="5.5.0.1", dst="1.1.0.1",
                              inner_src="1.1.0.1", inner_dst="5.5.0.1"))]),
        Case("icmp_error_no_flow_passes", f"{h}:113-120", ov, [
            Pkt(icmp4_err_frame("10.1.0.1", "10.2.0.1", "10.2.0.1", "10.1.0.1", 17), seeded_vni=100,
                expect=dict(done="Delivered", src="10.1.0.1", inner_src="10.2.0.1",
                            inner_dst="10.1.0.1")),
            Pkt(icmp4_err_frame("10.1.0.1", "10.2.0.1", "10.2.0.1", "10.1.0.1", 1), seeded_vni=100,
                expect=dict(done="Delivered"))]),
        Case("icmp_error_bad_checksum", f"{h}:77-88 (net/src/packet/icmp_err.rs:71-87)", ov, [
            Pkt(icmp4_err_frame("10.1.0.1", "10.2.0.1", "10.2.0.1", "10.1.0.1", bad_icmp_ck=True),
                seeded_vni=100, expect=dict(done="InvalidChecksum"))]),
        Case("icmp_error_incomplete", f"{h}:61-66,102-108 (net/src/packet/icmp_err.rs:178-228,"
             " net/src/flows/flow_key.rs:653-657)", ov, [
            Pkt(icmp4_err_frame("10.1.0.1", "10.2.0.1", "", "", inner=False), seeded_vni=100,
                expect=dict(done="IcmpErrorIncomplete")),
            Pkt(icmp4_err_frame("10.1.0.1", "10.2.0.1", "10.2.0.1", "10.1.0.1", 47), seeded_vni=100,
                expect=dict(done="IcmpErrorIncomplete")),
            Pkt(icmp4_err_frame("10.1.0.1", "10.2.0.1", "10.2.0.1", "10.1.0.1", -1), seeded_vni=100,
                expect=dict(done="IcmpErrorIncomplete"))]),
        # underlay: not the handler's business (overlay only); delivered with
        # its checksums refreshed (TTL -1)
        Case("icmp_error_underlay_delivered", f"{h}:184-194", ov, [
            Pkt(icmp4_err_frame("192.0.2.9", "203.0.113.5", "203.0.113.5", "192.0.2.9", ttl=64),
                expect=dict(done="Delivered", ttl=63, inner_src="203.0.113.5"))]),
    ]


def all_cases() -> List[Case]:
    return acl_cases() + ff_cases() + lpm_cases() + ttl_cases() + vxlan_qos_cases() + \
        parse_cases() + nat_cases() + pat_cases() + icmp_error_cases()


# ------------------------------------------------------------------ checks

def l3_of(frame: bytes) -> int:
    o = 14
    et = struct.unpack("!H", frame[12:14])[0]
    while et in (0x8100, 0x88A8, 0x9100):
        et = struct.unpack("!H", frame[o + 2:o + 4])[0]
        o += 4
    return o


def check(pkt: Pkt, out, frame_out: Optional[bytes]) -> List[str]:
    """Returns a list of mismatch descriptions (empty = pass)."""
    e, bad = pkt.expect, []
    done = A.DONE_NAMES[out["done"]] if out["done"] < A.DONE_COUNT else int(out["done"])
    if done != e["done"]:
        bad.append(f"done {done} != {e['done']}")
        return bad
    for k in ("acl", "dst_vni"):
        if k in e and int(out[k]) != e[k]:
            bad.append(f"{k} {int(out[k])} != {e[k]}")
    if "acl_rule" in e:
        got = None if out["acl_rule"] == 0xFFFFFFFF else int(out["acl_rule"])
        if got != e["acl_rule"]:
            bad.append(f"acl_rule {got} != {e['acl_rule']}")
    if "oif_in" in e and int(out["oif"]) not in e["oif_in"]:
        bad.append(f"oif {int(out['oif'])} not in {e['oif_in']}")
    if "fib_entry_in" in e and int(out["fib_entry"]) not in e["fib_entry_in"]:
        bad.append(f"fib_entry {int(out['fib_entry'])} not in {e['fib_entry_in']}")
    if frame_out is not None and ("inner_src" in e or "inner_dst" in e):
        # the embedded IPv4 header of an ICMPv4 error message
        o = l3_of(frame_out)
        eo = o + (frame_out[o] & 0xF) * 4 + 8
        isrc = str(ipaddress.IPv4Address(frame_out[eo + 12:eo + 16]))
        idst = str(ipaddress.IPv4Address(frame_out[eo + 16:eo + 20]))
        if "inner_src" in e and isrc != e["inner_src"]:
            bad.append(f"inner src {isrc} != {e['inner_src']}")
        if "inner_dst" in e and idst != e["inner_dst"]:
            bad.append(f"inner dst {idst} != {e['inner_dst']}")
    if frame_out is not None and any(k in e for k in ("ttl", "src", "dst", "outer_dscp",
                                                      "sport", "dport")):
        o = l3_of(frame_out)
        ver = frame_out[o] >> 4
        if ver == 4:
            tos, ttl = frame_out[o + 1], frame_out[o + 8]
            src = str(ipaddress.IPv4Address(frame_out[o + 12:o + 16]))
            dst = str(ipaddress.IPv4Address(frame_out[o + 16:o + 20]))
        else:
            tos = ((frame_out[o] & 0xF) << 4) | (frame_out[o + 1] >> 4)
            ttl = frame_out[o + 7]
            src = str(ipaddress.IPv6Address(frame_out[o + 8:o + 24]))
            dst = str(ipaddress.IPv6Address(frame_out[o + 24:o + 40]))
        if ver == 4 and ("sport" in e or "dport" in e):
            l4 = o + (frame_out[o] & 0xF) * 4
            sp, dp = struct.unpack("!HH", frame_out[l4:l4 + 4])
            if "sport" in e and sp != e["sport"]:
                bad.append(f"sport {sp} != {e['sport']}")
            if "dport" in e and dp != e["dport"]:
                bad.append(f"dport {dp} != {e['dport']}")
        if "ttl" in e and ttl != e["ttl"]:
            bad.append(f"ttl {ttl} != {e['ttl']}")
        if "src" in e and src != e["src"]:
            bad.append(f"src {src} != {e['src']}")
        if "dst" in e and dst != e["dst"]:
            bad.append(f"dst {dst} != {e['dst']}")
        if "outer_dscp" in e and (tos >> 2, tos & 3) != (e["outer_dscp"], e["outer_ecn"]):
            bad.append(f"outer dscp/ecn {(tos >> 2, tos & 3)} != {(e['outer_dscp'], e['outer_ecn'])}")
    return bad


# ------------------------------------------------------------------ runner

def run_case(case: Case, process) -> List[str]:
    """process(tables_ptr, buf, inp) -> out (dp_pkt_out_t array); buf is
    rewritten in place.  Returns mismatch descriptions."""
    from edgecase import pack_burst
    tb = case.tables()
    tp = tb.build()
    frames = [(p.frame, p.iif, A.IN_SEEDED_OVERLAY if p.seeded_vni else 0, p.seeded_vni)
              for p in case.packets]
    errs = []
    for k in range(case.passes):
        buf, inp = pack_burst(frames)
        out = process(tp, buf, inp)
        nxt = []
        for i, p in enumerate(case.packets):
            o = out[i]
            fo = None
            if o["done"] == A.DONE["Delivered"]:
                fo = bytes(buf[o["off"]:o["off"] + o["len"]])
            if k == case.passes - 1:
                errs += [f"{case.name}[{i}] ({case.ref}): {m}" for m in check(p, o, fo)]
                if fo is not None:
                    errs += [f"{case.name}[{i}]: {m}" for m in checksum_errors(fo)]
            nxt.append((fo if fo is not None else frames[i][0],) + frames[i][1:])
        frames = nxt
    return errs


def checksum_errors(frame: bytes) -> List[str]:
    """Checksum properties (net/src/checksum.rs:218-260): every IPv4 header
    and UDP/TCP checksum of a delivered frame validates (outer UDP of a VXLAN
    frame carries 0, net/src/packet/mod.rs:315-317)."""
    bad = []
    o = l3_of(frame)
    for _ in range(2):                     # outer, then the inner frame of VXLAN
        if len(frame) < o + 20:
            return bad
        ver = frame[o] >> 4
        if ver == 4:
            hl = (frame[o] & 0xF) * 4
            if P.csum_fold(P.sum16(frame[o:o + hl])) != 0:
                bad.append("ipv4 header checksum")
            proto, tl = frame[o + 9], struct.unpack("!H", frame[o + 2:o + 4])[0]
            l4o, src, dst = o + hl, frame[o + 12:o + 16], frame[o + 16:o + 20]
            pseudo = lambda n: src + dst + struct.pack("!BBH", 0, proto, n)  # noqa: E731
        elif ver == 6:
            proto = frame[o + 6]
            l4o, src, dst = o + 40, frame[o + 8:o + 24], frame[o + 24:o + 40]
            pseudo = lambda n: src + dst + struct.pack("!IxxxB", n, proto)  # noqa: E731
        else:
            return bad
        if proto == 17 and len(frame) >= l4o + 8:
            ulen = struct.unpack("!H", frame[l4o + 4:l4o + 6])[0]
            ck = struct.unpack("!H", frame[l4o + 6:l4o + 8])[0]
            dport = struct.unpack("!H", frame[l4o + 2:l4o + 4])[0]
            if dport == 4789 and ck == 0:
                o = l4o + 16 + 14
                continue
            if P.csum_fold(P.sum16(pseudo(ulen)) + P.sum16(frame[l4o:])) != 0:
                bad.append("udp checksum")
        elif proto == 6 and len(frame) >= l4o + 20:
            if P.csum_fold(P.sum16(pseudo(len(frame) - l4o)) + P.sum16(frame[l4o:])) != 0:
                bad.append("tcp checksum")
        elif proto == 1 and ver == 4 and len(frame) >= l4o + 8:
            # ICMPv4 over the whole message; an error message's embedded IPv4
            # header is refreshed too (net/src/headers/mod.rs:906-919)
            if P.csum_fold(P.sum16(frame[l4o:])) != 0:
                bad.append("icmp checksum")
            eo = l4o + 8
            if frame[l4o] in (3, 11, 12) and len(frame) >= eo + 20 and frame[eo] >> 4 == 4:
                ehl = (frame[eo] & 0xF) * 4
                if P.csum_fold(P.sum16(frame[eo:eo + ehl])) != 0:
                    bad.append("embedded ipv4 header checksum")
        return bad
    return bad
