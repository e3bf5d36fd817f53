"""Known-answer tests of the flow-filter classifier alone (dp_ff_classify,
FlowFilterContext::lookup / lookup_batch), transcribed from the reference's
own context tests (flow-filter/src/context/tests.rs:73-645).

Each overlay is lowered as the reference lowers it (RuleSet::from_overlay,
flow-filter/src/context/tables.rs:566-676) by tests/golden/natcombo.py's
lower(); a probe is a LookupInput (src VPC, the stage-1 GateVni -- None or a
VPC --, SourceGate, addresses, protocol, ports: `route_lookup`, tests.rs:45-
63, which takes the ports of a TCP / UDP header and none otherwise), and its
answer the LookupResult the test asserts:
  ("route", dst_vni, dst_nat, src_nat), ("srcmiss", dst_vni), ("dstmiss",),
or "miss" where the test only asserts that `route()` (tests.rs:28-41) gives
no Route.
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.tables import NAT_MASQUERADE, NAT_NONE, NAT_PORT_FORWARDING, NAT_STATIC
from golden.natcombo import Exp, Peering, lower, pwp

TCP, UDP, ICMP = 6, 17, 1
NONE, STATIC, MASQ, PF = NAT_NONE, NAT_STATIC, NAT_MASQUERADE, NAT_PORT_FORWARDING
UNGATED, PORTFWD_REPLY = 0, 1


def expose(*ips: str) -> Exp:             # expose / expose_multi (test_utils.rs:57-68)
    return Exp("plain", list(ips))


def expose_default() -> Exp:              # expose_default (:71-73)
    return Exp("default", [])


def expose_static(private: str, public: str) -> Exp:     # (:76-83)
    return Exp("static", [private], [public])


def expose_masquerade(private: str, public: str) -> Exp:  # (:86-93)
    return Exp("masq", [private], [public])


def expose_port_forwarding(private: str, pports, public: str, eports, proto=None) -> Exp:  # (:97-117)
    return Exp("pf", [pwp(private, *pports)], [pwp(public, *eports)], proto=proto)


@dataclass
class Probe:
    src_vni: int
    src: str
    dst: str
    proto: int = TCP
    ports: Optional[Tuple[int, int]] = (1234, 5678)
    dst_vpcd: Optional[int] = None
    gate: int = UNGATED
    want: object = "miss"


@dataclass
class Case:
    name: str
    ref: str
    peerings: Callable[[], List[Peering]]
    probes: List[Probe]


def routing_overlay():  # tests.rs:73-89
    return [Peering(100, [expose("1.0.0.0/24")], 200, [expose("5.0.0.0/24"), expose_default()]),
            Peering(100, [expose("1.0.0.0/24"), expose("2.0.0.0/24")], 300, [expose("6.0.0.0/24")])]


def nat_modes_overlay():  # tests.rs:204-227
    return [Peering(100, [expose("1.0.0.0/24"), expose_static("2.0.0.0/24", "20.0.0.0/24"),
                          expose_masquerade("3.0.0.0/24", "30.0.0.0/24")],
                    200, [expose("5.0.0.0/24"), expose_static("6.0.0.0/24", "60.0.0.0/24"), expose_default()])]


def dst_side_overlay():  # tests.rs:272-294
    return [Peering(100, [expose("10.0.0.0/24")],
                    200, [expose("90.0.0.0/24"), expose_masquerade("192.168.70.0/24", "70.0.0.0/24"),
                          expose_port_forwarding("192.168.80.5/32", (22, 22), "80.0.0.5/32", (2222, 2222), TCP)])]


def cases() -> List[Case]:
    t = "flow-filter/src/context/tests.rs"
    R = lambda d, dn, sn: ("route", d, dn, sn)  # noqa: E731
    return [
        Case("packet_allowed", f"{t}:92-116", routing_overlay, [
            Probe(100, "1.0.0.5", "5.0.0.10", want=R(200, NONE, NONE))]),
        Case("packet_filtered_when_source_prefix_unmatched", f"{t}:118-129", routing_overlay, [
            Probe(100, "9.9.9.9", "5.0.0.10")]),
        Case("packet_filtered_for_unknown_source_vpc", f"{t}:131-140", routing_overlay, [
            Probe(999, "1.0.0.5", "5.0.0.10")]),
        Case("default_remote_expose_is_catch_all", f"{t}:142-155", routing_overlay, [
            Probe(100, "1.0.0.5", "99.0.0.10", want=R(200, NONE, NONE))]),
        Case("overlapping_source_prefix_disambiguated_by_destination", f"{t}:157-194", routing_overlay, [
            Probe(100, "1.0.0.5", "5.0.0.10", want=("route", 200, None, None)),
            Probe(100, "1.0.0.5", "6.0.0.10", want=("route", 300, None, None)),
            Probe(100, "2.0.0.5", "6.0.0.10", want=("route", 300, None, None)),
            Probe(100, "2.0.0.5", "5.0.0.10")]),
        Case("nat_modes_source_and_destination", f"{t}:229-268", nat_modes_overlay, [
            Probe(100, "1.0.0.5", "5.0.0.10", want=R(200, NONE, NONE)),
            Probe(100, "2.0.0.5", "60.0.0.10", want=R(200, STATIC, STATIC)),
            Probe(100, "3.0.0.5", "5.0.0.10", want=R(200, NONE, MASQ)),
            Probe(100, "1.0.0.5", "60.0.0.10", want=R(200, STATIC, NONE)),
            Probe(100, "2.0.0.5", "5.0.0.10", want=R(200, NONE, STATIC)),
            Probe(100, "3.0.0.5", "99.0.0.10", want=R(200, NONE, MASQ))]),
        Case("dst_side_nat_modes", f"{t}:296-387", dst_side_overlay, [
            Probe(200, "192.168.70.1", "10.0.0.5", want=R(100, NONE, MASQ)),
            Probe(100, "10.0.0.5", "70.0.0.10", want=("dstmiss",)),
            Probe(100, "10.0.0.5", "70.0.0.10", dst_vpcd=200, want=R(200, MASQ, NONE)),
            Probe(100, "10.0.0.5", "80.0.0.5", ports=(1234, 2222), want=R(200, PF, NONE)),
            Probe(200, "192.168.80.5", "10.0.0.5", ports=(22, 1234), want=("srcmiss", 100)),
            Probe(200, "192.168.80.5", "10.0.0.5", ports=(22, 1234), gate=PORTFWD_REPLY, want=R(100, NONE, PF)),
            Probe(100, "10.0.0.5", "80.0.0.5", ports=(1234, 9999))]),
        Case("protocol_awareness", f"{t}:389-437", dst_side_overlay, [
            Probe(100, "10.0.0.5", "90.0.0.10", TCP, want=("route", 200, NONE, None)),
            Probe(100, "10.0.0.5", "90.0.0.10", UDP, want=("route", 200, NONE, None)),
            Probe(100, "10.0.0.5", "90.0.0.10", ICMP, None, want=("route", 200, NONE, None)),
            Probe(100, "10.0.0.5", "80.0.0.5", TCP, (1234, 2222), want=R(200, PF, NONE)),
            Probe(100, "10.0.0.5", "80.0.0.5", UDP, (1234, 2222)),
            Probe(100, "10.0.0.5", "80.0.0.5", ICMP, None)]),
        Case("source_default_expose_is_catch_all", f"{t}:439-462", lambda: [
            Peering(100, [expose("1.0.0.0/24"), expose_default()], 200, [expose("5.0.0.0/24")])], [
            Probe(100, "9.9.9.9", "5.0.0.10", want=R(200, NONE, NONE))]),
        Case("port_forwarding_any_protocol_matches_tcp_and_udp", f"{t}:464-494", lambda: [
            Peering(100, [expose("10.0.0.0/24")], 200,
                    [expose_port_forwarding("192.168.80.5/32", (22, 22), "80.0.0.5/32", (2222, 2222))])], [
            Probe(100, "10.0.0.5", "80.0.0.5", TCP, (1234, 2222), want=("route", 200, PF, None)),
            Probe(100, "10.0.0.5", "80.0.0.5", UDP, (1234, 2222), want=("route", 200, PF, None))]),
        Case("port_forwarding_and_masquerade_overlap", f"{t}:496-547", lambda: [
            Peering(100, [expose_masquerade("1.0.0.0/24", "100.0.0.0/24"),
                          expose_port_forwarding("1.0.0.27/32", (2000, 2001), "100.0.0.27/32", (3000, 3001), TCP)],
                    200, [expose("5.0.0.0/24")])], [
            Probe(100, "1.0.0.27", "5.0.0.10", ports=(2000, 5678), gate=PORTFWD_REPLY, want=R(200, NONE, PF)),
            Probe(100, "1.0.0.27", "5.0.0.10", ports=(2000, 5678), want=R(200, NONE, MASQ))]),
        Case("ipv6_lookup", f"{t}:549-575", lambda: [
            Peering(100, [expose("2001:db8::/32")], 200, [expose("2001:db9::/32")])], [
            Probe(100, "2001:db8::1", "2001:db9::1", want=("route", 200, None, None)),
            Probe(100, "2001:db8::1", "2001:dba::1")]),
        Case("discrepancy_overlapping_contiguous_prefixes", f"{t}:577-654", lambda: [
            Peering(100, [expose("10.0.2.0/24")], 200, [expose("20.0.0.0/24")]),
            Peering(100, [expose("10.0.2.2/32", "10.0.2.3/32")], 300, [expose("30.0.0.0/24")])], [
            Probe(100, "10.0.2.2", "30.0.0.1", ports=(9999, 80), want=R(300, NONE, NONE)),
            Probe(300, "30.0.0.1", "10.0.2.2", ports=(80, 9999), want=R(100, NONE, NONE))]),
        # reference_and_dpdk_backends_agree (:656-845): its probes, whose
        # answers the test pins only as "both backends agree"; here the
        # values are the restatement's, GPU == oracle
        Case("backends_agree_probes", f"{t}:656-845", lambda: [
            Peering(100, [expose("1.0.0.0/24"), expose_static("2.0.0.0/24", "20.0.0.0/24"),
                          expose_masquerade("3.0.0.0/24", "30.0.0.0/24")],
                    200, [expose("5.0.0.0/24"), expose_default()]),
            Peering(100, [expose("2001:db8::/32")], 300, [expose("2001:db9::/32")])], [
            Probe(100, "1.0.0.5", "5.0.0.10", TCP, want=R(200, NONE, NONE)),
            Probe(100, "1.0.0.5", "5.0.0.10", UDP, want=R(200, NONE, NONE)),
            Probe(100, "1.0.0.5", "5.0.0.10", ICMP, None, want=R(200, NONE, NONE)),
            Probe(100, "2.0.0.5", "5.0.0.10", want=R(200, NONE, STATIC)),
            Probe(100, "1.0.0.5", "99.0.0.10", want=R(200, NONE, NONE)),
            Probe(100, "9.9.9.9", "5.0.0.10", want=("srcmiss", 200)),
            Probe(100, "1.0.0.5", "6.6.6.6", want=R(200, NONE, NONE)),
            Probe(999, "1.0.0.5", "5.0.0.10", want=("dstmiss",)),
            Probe(100, "3.0.0.5", "5.0.0.10", want=R(200, NONE, MASQ)),
            Probe(200, "5.0.0.10", "30.0.0.5", ports=(5678, 1234), want=("dstmiss",)),
            Probe(200, "5.0.0.10", "30.0.0.5", ICMP, None, want=("dstmiss",)),
            Probe(100, "2001:db8::1", "2001:db9::1", want=R(300, NONE, NONE)),
            Probe(100, "2001:db8::1", "2001:dba::1", want=("dstmiss",)),
            Probe(100, "1.0.0.5", "2001:db9::1", want=("dstmiss",))]),
    ]


def inputs(probes: List[Probe]) -> np.ndarray:
    out = np.zeros(len(probes), A.FF_INPUT)
    for i, p in enumerate(probes):
        s, d = ipaddress.ip_address(p.src), ipaddress.ip_address(p.dst)
        out[i]["src_vni"] = p.src_vni
        out[i]["dst_vni"] = p.dst_vpcd or 0
        out[i]["src_family"], out[i]["dst_family"] = s.version, d.version
        out[i]["proto"] = p.proto
        out[i]["gate"] = p.gate
        if p.ports is not None:
            out[i]["sport"], out[i]["dport"] = p.ports
        out[i]["src"][:len(s.packed)] = np.frombuffer(s.packed, np.uint8)
        out[i]["dst"][:len(d.packed)] = np.frombuffer(d.packed, np.uint8)
    return out


def check(case: Case, res: np.ndarray) -> List[str]:
    errs = []
    names = {A.FF_ROUTE: "route", A.FF_SOURCE_MISS: "srcmiss", A.FF_DESTINATION_MISS: "dstmiss"}
    for p, r in zip(case.probes, res):
        got = names[int(r["outcome"])]
        w = p.want
        tag = f"{case.name}: {p.src} -> {p.dst} from {p.src_vni}"
        if w == "miss":
            if got == "route":
                errs.append(f"{tag}: a route, want a miss")
            continue
        if got != w[0]:
            errs.append(f"{tag}: {got}, want {w[0]}")
            continue
        if got in ("route", "srcmiss") and int(r["dst_vni"]) != w[1]:
            errs.append(f"{tag}: dst VPC {int(r['dst_vni'])}, want {w[1]}")
        if got == "route":
            if w[2] is not None and int(r["dst_nat"]) != w[2]:
                errs.append(f"{tag}: dst NAT {int(r['dst_nat'])}, want {w[2]}")
            if w[3] is not None and int(r["src_nat"]) != w[3]:
                errs.append(f"{tag}: src NAT {int(r['src_nat'])}, want {w[3]}")
    return errs


def tables(case: Case):
    return lower(case.peerings())
