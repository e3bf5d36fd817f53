"""Known-answer tests of masquerade, transcribed from
the reference's own Masquerade tests (nat/src/masquerade/test.rs).

The reference tests run the IcmpErrorHandler, FlowLookup, a test flow filter
(it sets the destination VPC of every packet from a fixed peer map; the test
packets are marked for masquerade by hand) and Masquerade, packet by packet,
with the allocator updated by hand in between (update_nat_allocator).  Here
each packet is a burst of its own through the whole path, with flow-filter
tables that play that test flow filter: every VPC's packets get the peer as
destination and the masquerade requirement (a local rule of 0/0 with
NatRequirement::Masquerade), and a peer's remote rule exists both ungated and
gated on the VPC (the gated one is what revalidating an outdated reply flow
asks, flow-filter/src/context/tables.rs:583-622).  The one test that runs the
reference's real flow filter (test_full_config_unidirectional_nat_
overlapping_destination) gets the real lowering instead: the masquerade
public range gated on its VPC.  An allocator update is a publish of the next
generation (dp_tables_publish runs update_nat_allocator for the attached flow
table); the flow-filter tables stay as they were, as the test flow filter
does.  The allocator is the reference's deterministic one
(set_randomize(false)); steps that assert only what the reference asserts are
KATs, the exact tuples (port 1024: the first block past the IANA well-known
range) are the restatement's, compared between the oracle and the GPU.
"""
from __future__ import annotations

import ipaddress
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.tables import NAT_MASQUERADE, NAT_NONE, TablesBuilder
from edgecase import pack_burst
from golden.kat import IF_MAC, NH_MAC, OIF_MAC, PEER_MAC, icmp4_err_frame
from golden.pfkat import GpuRunner as _PfGpuRunner, fields
import pktgen as P

TB = TablesBuilder
SEC = 1_000_000_000
MIN = 60 * SEC
FIN, SYN, RST, PSH, ACK = 0x01, 0x02, 0x04, 0x08, 0x10
V1, V2, V3, V4 = 100, 200, 300, 400


def excl(net: str, *holes: str) -> List[str]:
    """Prefix::subtract: `net` without the holes (VpcExpose not / not_as)."""
    out = [ipaddress.ip_network(net)]
    for h in holes:
        hn = ipaddress.ip_network(h)
        nxt = []
        for n in out:
            nxt += list(n.address_exclude(hn)) if hn.subnet_of(n) else [n]
        out = nxt
    return [str(n) for n in sorted(out)]


# ---------------------------------------------------------------------------
# overlays: the masquerade exposes of each test config (test.rs:146-471)
# ---------------------------------------------------------------------------
def overlay_4vpcs():  # build_overlay_4vpcs (test.rs:146-283)
    return [
        (V1, V2, ["1.1.0.0/16"], ["10.12.0.0/16"], 60),                       # expose121
        (V1, V2, ["1.2.0.0/16"], ["10.98.128.0/17", "10.99.0.0/17"], 0),      # expose122
        (V1, V2, ["1.3.0.0/24"], ["10.100.0.0/24"], 0),                       # expose123
        (V1, V3, ["1.1.0.0/16"], ["3.3.0.0/16"], 0),                          # expose131
        (V1, V3, ["1.2.0.0/16"], excl("3.1.0.0/16", "3.1.128.0/17") + ["3.2.0.0/17"], 0),
        (V1, V4, ["1.1.0.0/16"], ["4.4.0.0/16"], 0),                          # expose141
        (V2, V4, excl("2.4.0.0/16", "2.4.1.0/24"), excl("44.0.0.0/16", "44.0.200.0/24"), 0),
        (V3, V4, ["192.168.100.0/24"], ["34.34.34.0/24"], 0),                 # expose341
    ]


OVERLAYS = {
    "4vpcs": overlay_4vpcs,
    "2vpcs": lambda: [(V1, V2, ["1.1.0.0/16"], ["2.2.0.0/16"], 0)],
    "2vpcs_modified": lambda: [(V1, V2, ["1.1.0.0/16"], ["4.4.0.0/16"], 0)],
    "shared": lambda: [(V1, V3, ["1.1.0.0/16"], ["2.2.0.0/16"], 0),
                       (V2, V3, ["1.1.0.0/16"], ["4.4.0.0/16"], 0)],
    "shared_extended": lambda: [(V1, V3, ["1.1.0.0/16"], ["2.2.0.0/16"], 0),
                                (V1, V3, ["1.9.0.0/16"], ["9.9.0.0/16"], 0),
                                (V2, V3, ["1.1.0.0/16"], ["4.4.0.0/16"], 0)],
    "shared_narrowed": lambda: [(V1, V3, ["1.7.0.0/16"], ["2.2.0.0/16"], 0),
                                (V2, V3, ["1.1.0.0/16"], ["4.4.0.0/16"], 0)],
    "shared_v2_only": lambda: [(V2, V3, ["1.1.0.0/16"], ["4.4.0.0/16"], 0)],
    "none": lambda: [],
    "overlap": lambda: [(V1, V2, ["1.0.0.0/24"], ["2.0.0.0/24"], 0),
                        (V3, V2, ["1.0.0.0/24"], ["2.0.0.0/24"], 0)],
}

# the test flow filter's peer map, per scenario family: (src VPC, dst VPC)
PEERS = {
    "2vpcs": [(V1, V2), (V2, V1)],
    "shared": [(V1, V3), (V2, V3)],
}


def world(overlay: str, genid: int, peers: Optional[list] = None, real_ff: bool = False,
          routes: Optional[Dict[int, List[tuple]]] = None) -> TablesBuilder:
    t = TB(genid=genid)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    for v in (V1, V2, V3, V4):
        t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
        # (empty) static NAT tables: the ICMP error handler asks for static NAT
        t.add_nat_table(0, v, 0, [])
    for (s, d, priv, pub, idle) in OVERLAYS[overlay]():
        t.add_masquerade(s, d, priv, pub, idle_timeout_s=idle)
    if real_ff:
        # the reference's lowering of build_overlay_3vpcs_unidirectional_nat_
        # overlapping_addr (flow-filter/src/context/tables.rs:583-662)
        t.add_ff_remote(V1, "5.0.0.0/24", V2)
        t.add_ff_local(V1, V2, "1.0.0.0/24", NAT_MASQUERADE)
        t.add_ff_remote(V3, "5.0.0.0/24", V2)
        t.add_ff_local(V3, V2, "1.0.0.0/24", NAT_MASQUERADE)
        t.add_ff_remote(V2, "2.0.0.0/24", V1, NAT_MASQUERADE, gate_vni=V1)
        t.add_ff_remote(V2, "2.0.0.0/24", V3, NAT_MASQUERADE, gate_vni=V3)
        t.add_ff_local(V2, V1, "5.0.0.0/24")
        t.add_ff_local(V2, V3, "5.0.0.0/24")
    elif routes:
        # destination prefixes -> VPC (check_packet sets the destination VPC)
        for s, lst in routes.items():
            for (pfx, d) in lst:
                t.add_ff_remote(s, pfx, d)
                t.add_ff_remote(s, pfx, d, gate_vni=d)
            for d in sorted({d for _, d in lst}):
                t.add_ff_local(s, d, "0.0.0.0/0", NAT_MASQUERADE)
    else:
        for (s, d) in peers:
            t.add_ff_remote(s, "0.0.0.0/0", d)
            t.add_ff_remote(s, "0.0.0.0/0", d, gate_vni=d)
            t.add_ff_local(s, d, "0.0.0.0/0", NAT_MASQUERADE)
    return t


# ---------------------------------------------------------------------------
# packets (net/src/packet/test_utils.rs)
# ---------------------------------------------------------------------------
def l4_frame(src: str, dst: str, proto: int, sport: int, dport: int, flags: int = 0) -> bytes:
    if proto == 6:
        body = P.tcp(sport, dport, b"", P.pseudo4(src, dst, 6, 20), flags=flags)
    else:
        body = P.udp(sport, dport, b"", P.pseudo4(src, dst, 17, 8))
    return P.eth(IF_MAC, PEER_MAC, 0x0800) + P.ipv4(src, dst, proto, len(body)) + body


def echo_frame(src: str, dst: str, ident: int, reply: bool = False, seq: int = 0) -> bytes:
    """build_test_icmp4_echo (test_utils.rs)"""
    body = P.icmp4(0 if reply else 8, 0, struct.pack("!HH", ident, seq), b"")
    return P.eth(IF_MAC, PEER_MAC, 0x0800) + P.ipv4(src, dst, 1, len(body)) + body


@dataclass
class Pkt:
    frame: bytes
    vni: int


def tcp_from(vni: int, src: str, sport: int, syn: bool) -> Pkt:  # tcp_from (test.rs:474-487)
    return Pkt(l4_frame(src, "3.3.3.1", 6, sport, 80, SYN if syn else 0), vni)


def tcp_masq(flags: int = 0) -> Pkt:  # tcp_packet_to_masquerade (test.rs:1553-1564)
    return Pkt(l4_frame("1.1.0.1", "3.3.3.1", 6, 4321, 80, flags), V1)


def out_fields(fr: bytes) -> dict:
    f = fields(fr)
    if f["proto"] == 1:
        ihl = (fr[14] & 15) * 4
        f["ident"] = struct.unpack("!H", fr[14 + ihl + 4:14 + ihl + 6])[0]
        if fr[14 + ihl] in (3, 11, 12):  # an error: its embedded packet
            e = 14 + ihl + 8
            eihl = (fr[e] & 15) * 4
            f["isrc"] = str(ipaddress.ip_address(fr[e + 12:e + 16]))
            f["idst"] = str(ipaddress.ip_address(fr[e + 16:e + 20]))
            f["iid"], f["iseq"] = struct.unpack("!HH", fr[e + eihl + 4:e + eihl + 8])
            # (an embedded TCP / UDP header: its ports)
            f["isport"], f["idport"] = struct.unpack("!HH", fr[e + eihl:e + eihl + 4])
    return f


REPLY = "reply"    # build_reply (test.rs:1608-1638) of the previous delivered output


def reply(flags_set: int = 0, flags_clear: int = 0, udp: bool = False):
    return (REPLY, flags_set, flags_clear)


@dataclass
class Step:
    pkt: object                                 # Pkt or a reply(...) tuple
    expect: Dict = field(default_factory=dict)
    publish: Optional[tuple] = None             # (overlay, genid) published first
    sweep: bool = False                         # the flow timers up to the clock first
    advance: int = SEC
    save: Optional[str] = None                  # remember this output's (src, sport)


@dataclass
class Scenario:
    name: str
    ref: str
    overlay: str
    steps: List[Step]
    peers: Optional[list] = None
    real_ff: bool = False
    routes: Optional[dict] = None
    # (overlay name, genid) -> TablesBuilder, instead of world(): the NAT
    # composition scenarios (tests/golden/natcombo.py) lower whole overlays
    build: Optional[Callable[[str, int], TablesBuilder]] = None


def establish() -> List[Step]:  # establish_tcp_connection (test.rs:1651-1687)
    return [Step(tcp_masq(SYN), dict(done="Delivered")),
            Step(reply(), dict(flow=True, status=A.FLOW_ACTIVE, nat_status=A.NFS_TWO_WAY)),
            Step(tcp_masq(ACK), dict(done="Delivered", status=A.FLOW_ACTIVE,
                                     nat_status=A.NFS_ESTABLISHED, expires_in=120 * SEC - 5 * SEC,
                                     related_expires_in=120 * SEC - 5 * SEC))]


def scenarios() -> List[Scenario]:
    t = "nat/src/masquerade/test.rs"
    two = PEERS["2vpcs"]
    sh = PEERS["shared"]
    sc = []
    # test_full_config (:546-627): the first config; the reference runs a
    # second update against a flow table the NF does not use, which has no
    # counterpart here
    routes4 = {V1: [("10.201.0.0/16", V2), ("9.9.9.9/32", V2), ("3.3.3.0/24", V3), ("4.5.0.0/16", V4)],
               V2: [("10.12.0.0/16", V1), ("10.98.0.0/15", V1), ("44.4.0.0/16", V4)],
               V3: [("1.1.0.0/16", V1), ("4.4.0.0/24", V4)],
               V4: [("2.4.0.0/16", V2)]}
    sc.append(Scenario("full_config", f"{t}:546-627", "4vpcs", [
        Step(Pkt(l4_frame("8.8.8.8", "9.9.9.9", 17, 9998, 443), V1), dict(done="Filtered")),
        Step(Pkt(l4_frame("1.1.2.3", "10.201.201.18", 17, 9998, 443), V1),
             dict(done="Delivered", src="10.12.0.0", dst="10.201.201.18", idle=60)),
        Step(reply(udp=True), dict(done="Delivered", src="10.201.201.18", dst="1.1.2.3", sport=443,
                                   dport=9998, idle=60)),
        # the other exposes and peers of the config (restatement-derived tuples)
        Step(Pkt(l4_frame("1.2.7.7", "10.201.201.18", 6, 5000, 80, SYN), V1),
             dict(done="Delivered", src="10.98.128.0", sport=1024)),
        Step(Pkt(l4_frame("1.3.0.9", "10.201.202.1", 17, 5000, 53), V1),
             dict(done="Delivered", src="10.100.0.0", sport=1024)),
        Step(Pkt(l4_frame("1.1.2.3", "3.3.3.7", 17, 9998, 443), V1),
             dict(done="Delivered", src="3.3.0.0", sport=1024)),
        Step(Pkt(l4_frame("1.2.9.9", "3.3.3.7", 17, 9998, 443), V1),
             dict(done="Delivered", src="3.1.0.0", sport=1024)),
        Step(Pkt(l4_frame("1.1.2.3", "4.5.6.7", 17, 9998, 443), V1),
             dict(done="Delivered", src="4.4.0.0", sport=1024)),
        Step(Pkt(l4_frame("2.4.5.6", "44.4.1.1", 17, 7000, 443), V2),
             dict(done="Delivered", src="44.0.0.0", sport=1024)),
        Step(Pkt(l4_frame("2.4.1.7", "44.4.1.1", 17, 7000, 443), V2), dict(done="Filtered")),
        Step(Pkt(l4_frame("192.168.100.9", "4.4.0.1", 17, 7000, 443), V3),
             dict(done="Delivered", src="34.34.34.0", sport=1024)),
        Step(Pkt(l4_frame("1.1.2.3", "10.201.201.18", 17, 9999, 443), V1),
             dict(done="Delivered", src="10.12.0.0", sport=1025)),
    ], routes=routes4))
    # test_icmp_echo_nat (:788-883)
    sc.append(Scenario("icmp_echo_nat", f"{t}:788-883", "2vpcs", [
        Step(Pkt(echo_frame("8.8.8.8", "9.9.9.9", 1337), V1), dict(done="Filtered")),
        Step(Pkt(echo_frame("1.1.2.3", "3.3.3.3", 1337), V1),
             dict(done="Delivered", src="2.2.0.0", dst="3.3.3.3", ident_mod256=0, ident=0), save="echo"),
        Step(reply(), dict(done="Delivered", src="3.3.3.3", dst="1.1.2.3", ident=1337)),
        Step(Pkt(echo_frame("1.1.2.3", "3.3.3.3", 1337), V1),
             dict(done="Delivered", src="2.2.0.0", same_ident="echo")),
        Step(Pkt(echo_frame("1.1.2.3", "3.3.3.3", 0), V1),
             dict(done="Delivered", src="2.2.0.0", ident_next="echo")),
    ], peers=two))
    # test_icmp_error_nat (:955-1076)
    err0 = icmp4_err_frame("1.2.2.18", "2.2.0.0", "2.2.0.0", "3.3.3.3", 1, 1337, 0)
    sc.append(Scenario("icmp_error_nat", f"{t}:955-1076", "2vpcs", [
        Step(Pkt(err0, V2), dict(done="Delivered", src="1.2.2.18", dst="2.2.0.0", isrc="2.2.0.0",
                                 idst="3.3.3.3", iid=1337, iseq=0)),
        Step(Pkt(echo_frame("1.1.2.3", "3.3.3.3", 1337), V1),
             dict(done="Delivered", src="2.2.0.0", dst="3.3.3.3", ident_mod256=0), save="echo"),
        Step(("icmp_err_for", "echo"), dict(done="Delivered", src="1.2.2.18", dst="1.1.2.3",
                                           isrc="1.1.2.3", idst="3.3.3.3", iid=1337, iseq=0)),
    ], peers=two))
    # test_default_expose (:1104-1190): a default expose of the peer is a /0 rule
    sc.append(Scenario("default_expose", f"{t}:1104-1190", "2vpcs", [
        Step(Pkt(l4_frame("1.1.0.1", "3.3.3.3", 17, 9999, 443), V1),
             dict(done="Delivered", src="2.2.0.0", dst="3.3.3.3")),
        Step(reply(udp=True), dict(done="Delivered", src="3.3.3.3", dst="1.1.0.1", sport=443, dport=9999)),
        Step(Pkt(l4_frame("1.1.0.1", "10.11.12.13", 17, 9999, 443), V1),
             dict(done="Delivered", src="2.2.0.0", dst="10.11.12.13")),
        Step(reply(udp=True), dict(done="Delivered", src="10.11.12.13", dst="1.1.0.1", sport=443,
                                   dport=9999)),
    ], routes={V1: [("3.3.3.0/24", V2), ("0.0.0.0/0", V2)], V2: [("2.2.0.0/16", V1)]}))
    # test_full_config_unidirectional_nat_overlapping_destination (:1302-1551),
    # with the reference's real flow filter
    sc.append(Scenario("unidirectional_overlapping_destination", f"{t}:1302-1551", "overlap", [
        # no flow yet: the masquerade public range answers only a revalidation
        Step(Pkt(l4_frame("5.0.0.5", "2.0.0.0", 17, 443, 1024), V2), dict(done="Filtered")),
        Step(Pkt(l4_frame("1.0.0.18", "5.0.0.5", 17, 9998, 443), V1),
             dict(done="Delivered", src="2.0.0.0", dst="5.0.0.5", sport_lowport=True, dport=443,
                  dst_vni=V2, sport=1024)),
        Step(reply(udp=True), dict(done="Delivered", src="5.0.0.5", dst="1.0.0.18", sport=443,
                                   dport=9998, dst_vni=V1)),
        Step(Pkt(l4_frame("5.0.0.5", "2.0.0.0", 17, 443, 1024), V2),
             dict(done="Delivered", dst="1.0.0.18", dport=9998, dst_vni=V1)),
        Step(Pkt(l4_frame("1.0.0.18", "5.0.0.5", 17, 9998, 443), V3),
             dict(done="Delivered", src="2.0.0.0", dst="5.0.0.5", sport_mod256=1, dst_vni=V2,
                  sport=1025)),
        Step(Pkt(l4_frame("5.0.0.5", "2.0.0.0", 17, 443, 1024), V2),
             dict(done="Delivered", dst="1.0.0.18", dport=9998, dst_vni=V1)),
    ], real_ff=True))
    sc.append(Scenario("tcp_establish", f"{t}:1689-1696", "2vpcs", establish() + [
        Step(None, dict(active=2))], peers=two))
    sc.append(Scenario("check", f"{t}:1698-1738", "2vpcs", establish() + [
        Step(tcp_masq(), dict(masq=A.PF_SRC_NAT)),
        Step(reply(), dict(masq=A.PF_DST_NAT, nat_status=A.NFS_ESTABLISHED, status=A.FLOW_ACTIVE,
                           src="3.3.3.1", dst="1.1.0.1", sport=80, dport=4321)),
        Step(None, dict(active=2))], peers=two))
    sc.append(Scenario("tcp_reset", f"{t}:1740-1774", "2vpcs", establish() + [
        Step(tcp_masq()),
        Step(reply(RST, ACK), dict(masq=A.PF_DST_NAT, nat_status=A.NFS_RESET, status=A.FLOW_CANCELLED,
                                   src="3.3.3.1", dst="1.1.0.1", sport=80, dport=4321)),
        Step(None, dict(active=0, flows=0), sweep=True)], peers=two))
    sc.append(Scenario("tcp_close_client", f"{t}:1776-1822", "2vpcs", establish() + [
        Step(tcp_masq(FIN), dict(nat_status=A.NFS_C_CLOSING), save="closing"),
        Step(reply(0, FIN), dict(nat_status=A.NFS_C_HALF_CLOSE)),
        Step(("reply_of", "closing", FIN, 0), dict(nat_status=A.NFS_LAST_ACK)),
        Step(tcp_masq(ACK), dict(nat_status=A.NFS_CLOSED)),
    ], peers=two))
    sc.append(Scenario("tcp_close_server", f"{t}:1824-1873", "2vpcs", establish() + [
        Step(tcp_masq(), save="out"),
        Step(("reply_of", "out", FIN, 0), dict(nat_status=A.NFS_S_CLOSING)),
        Step(tcp_masq(ACK), dict(nat_status=A.NFS_S_HALF_CLOSE)),
        Step(tcp_masq(FIN), dict(nat_status=A.NFS_LAST_ACK)),
        Step(("reply_of", "out", 0, FIN), dict(nat_status=A.NFS_CLOSED)),
    ], peers=two))
    sc.append(Scenario("reconfig_keep_flow", f"{t}:1875-1909", "2vpcs", establish() + [
        Step(tcp_masq()),
        Step(reply(), dict(nat_status=A.NFS_ESTABLISHED, status=A.FLOW_ACTIVE, genid=1)),
        Step(tcp_masq(), dict(nat_status=A.NFS_ESTABLISHED, status=A.FLOW_ACTIVE, genid=2),
             publish=("2vpcs", 2)),
        Step(None, dict(active=2))], peers=two))
    sc.append(Scenario("reconfig_two_vpcs_sharing_a_private_prefix", f"{t}:1911-1965", "shared", [
        Step(tcp_from(V1, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, True)),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(src_net="2.2.0.0/16", genid=1), save="v1"),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(src_net="4.4.0.0/16", genid=1), save="v2"),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(same="v1", genid=2), publish=("shared", 2)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(same="v2", genid=2)),
        Step(None, dict(active=4))], peers=sh))
    sc.append(Scenario("reconfig_carries_flows_into_a_new_allocator", f"{t}:1967-2023", "shared", [
        Step(tcp_from(V1, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, True)),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(src_net="2.2.0.0/16"), save="v1"),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(src_net="4.4.0.0/16"), save="v2"),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(same="v1"), publish=("shared_extended", 2)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(same="v2")),
        Step(tcp_from(V1, "1.1.0.1", 5555, True)),
        Step(tcp_from(V1, "1.1.0.1", 5555, False), dict(differs=("v1", "v2"), genid=2)),
    ], peers=sh))
    sc.append(Scenario("reconfig_drops_a_flow_whose_peering_is_gone", f"{t}:2025-2083", "shared", [
        Step(tcp_from(V1, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), save="v2"),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(done="Filtered"), publish=("shared_v2_only", 2)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(same="v2")),
    ], peers=sh))
    sc.append(Scenario("reconfig_drops_a_flow_whose_source_is_no_longer_exposed", f"{t}:2085-2122",
                       "shared", [
        Step(tcp_from(V1, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), save="v2"),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(done="Filtered"), publish=("shared_narrowed", 2)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(same="v2")),
    ], peers=sh))
    sc.append(Scenario("reconfig_without_masquerade_drops_every_flow", f"{t}:2124-2150", "shared", [
        Step(tcp_from(V1, "1.1.0.1", 4321, True)),
        Step(tcp_from(V2, "1.1.0.1", 4321, True)),
        Step(tcp_from(V1, "1.1.0.1", 4321, False), dict(done="NatFailure"), publish=("none", 2)),
        Step(tcp_from(V2, "1.1.0.1", 4321, False), dict(done="NatFailure")),
        Step(None, dict(active=0), sweep=True),
    ], peers=sh))
    sc.append(Scenario("reconfig_drop_flow", f"{t}:2152-2188", "2vpcs", establish() + [
        Step(tcp_masq()),
        Step(reply(), dict(nat_status=A.NFS_ESTABLISHED, status=A.FLOW_ACTIVE, genid=1)),
        Step(tcp_masq(), dict(nat_status=A.NFS_ESTABLISHED, not_status=A.FLOW_ACTIVE, genid=1,
                              done="Filtered"), publish=("2vpcs_modified", 2)),
        Step(None, dict(active=0), sweep=True)], peers=two))
    # test_genid_updated_on_reconfig (:2190-2217): the allocator's generation,
    # seen as the genid of the flows it creates
    sc.append(Scenario("genid_updated_on_reconfig", f"{t}:2190-2217", "2vpcs", [
        Step(Pkt(l4_frame("1.1.0.1", "3.3.3.1", 17, 1000, 53), V1), dict(genid=1)),
        Step(Pkt(l4_frame("1.1.0.1", "3.3.3.1", 17, 1001, 53), V1), dict(genid=2), publish=("2vpcs", 2)),
        Step(Pkt(l4_frame("1.1.0.1", "3.3.3.1", 17, 1002, 53), V1), dict(genid=3, src="4.4.0.0"),
             publish=("2vpcs_modified", 3)),
    ], peers=two))
    return sc


# ---------------------------------------------------------------------------
# runners
# ---------------------------------------------------------------------------
class OracleRunner:
    """The oracle as one device: tables, a flow table, the flow clock.  A
    publish runs update_nat_allocator on the flow table (dpo_flows_sync)."""

    def __init__(self, **_):
        from oracle.pyoracle import Oracle, OracleFlows
        self._Oracle = Oracle
        self.fl = OracleFlows()
        self.tabs = None
        self.keep = []

    def publish(self, builder: TablesBuilder):
        self.keep.append(builder)
        self.tabs = self._Oracle(builder.build(), prev=self.tabs)
        self.fl.sync(self.tabs)

    def set_clock(self, ns: int):
        self.fl.set_clock(ns)

    def burst(self, buf, inp):
        res, _ = self.tabs.process_flows(buf, inp, self.fl)
        return res

    def get(self, refs):
        return self.fl.get(np.asarray(refs, np.uint64))

    def count(self):
        return self.fl.count()

    def sweep(self, now):
        return self.fl.sweep(now)

    def lookup(self, keys):
        return self.fl.lookup(keys)


GpuRunner = _PfGpuRunner


def run_scenario(s: Scenario, r, on_step=None) -> List[str]:
    errs: List[str] = []
    now = 0
    mk = s.build or (lambda ov, g: world(ov, g, s.peers, s.real_ff, s.routes))
    r.publish(mk(s.overlay, 1))
    last = None            # (fields, dst_vni) of the previous delivered output
    saved: Dict[str, tuple] = {}
    for i, st in enumerate(s.steps):
        now += st.advance
        r.set_clock(now)
        if st.publish is not None:
            r.publish(mk(st.publish[0], st.publish[1]))
        if st.sweep:
            r.sweep(now)
        tag = f"{s.name} step {i}"
        e = st.expect
        pkt = st.pkt
        if pkt is None:   # flow-table checks only
            ln, act = r.count()
            if "active" in e and act != e["active"]:
                errs.append(f"{tag}: active flows {act} != {e['active']}")
            if "flows" in e and ln != e["flows"]:
                errs.append(f"{tag}: flows {ln} != {e['flows']}")
            continue
        if callable(pkt):  # built from what earlier steps delivered
            pkt = pkt(saved, last)
        if isinstance(pkt, tuple) and pkt[0] in (REPLY, "reply_of"):
            if pkt[0] == REPLY:
                base, fset, fclr = last, pkt[1], pkt[2]
            else:
                base, fset, fclr = saved[pkt[1]][2], pkt[2], pkt[3]
            o, dvni = base
            fl = o["flags"]
            if o["proto"] == 6:
                if fl & SYN and fl & ACK:
                    fl &= ~SYN
                fl |= ACK
                fl = (fl | fset) & ~fclr
            if o["proto"] == 1:
                fr = echo_frame(o["dst"], o["src"], o["ident"], reply=True)
            else:
                fr = l4_frame(o["dst"], o["src"], o["proto"], o["dport"], o["sport"], fl)
            pkt = Pkt(fr, dvni)
        elif isinstance(pkt, tuple) and pkt[0] == "icmp_err_for":
            o = saved[pkt[1]][2][0]
            pkt = Pkt(icmp4_err_frame("1.2.2.18", o["src"], o["src"], o["dst"], 1, o["ident"], 0), V2)
        buf, inp = pack_burst([(pkt.frame, 1, A.IN_SEEDED_OVERLAY, pkt.vni)])
        res = r.burst(buf, inp)
        o = res[0]
        done = A.DONE_NAMES[o["done"]] if o["done"] < A.DONE_COUNT else str(o["done"])
        out = None
        if done == "Delivered":
            out = out_fields(buf[o["off"]:o["off"] + o["len"]].tobytes())
            last = (out, int(o["dst_vni"]))
            if st.save:
                saved[st.save] = (out["src"], out.get("ident", out["sport"]), last)
        ref = int(o["flow_ref"])
        info = r.get([ref])[0] if ref != A.FLOW_NONE else None
        if on_step:
            on_step(i, res, buf, info)
        if "done" in e and done != e["done"]:
            errs.append(f"{tag}: done {done} != {e['done']}")
        for k in ("src", "dst", "sport", "dport", "ident", "isrc", "idst", "iid", "iseq", "isport",
                  "idport"):
            if k in e and (out is None or out.get(k) != e[k]):
                errs.append(f"{tag}: {k} {None if out is None else out.get(k)} != {e[k]}")
        if "dst_vni" in e and int(o["dst_vni"]) != e["dst_vni"]:
            errs.append(f"{tag}: dst_vni {int(o['dst_vni'])} != {e['dst_vni']}")
        if out is not None:
            if "not_sport" in e and out["sport"] == e["not_sport"]:
                errs.append(f"{tag}: sport {out['sport']} is the excluded {e['not_sport']}")
            if "ident_mod256" in e and out["ident"] % 256 != e["ident_mod256"]:
                errs.append(f"{tag}: identifier {out['ident']} not the first of a block")
            if "sport_mod256" in e and out["sport"] % 256 != e["sport_mod256"]:
                errs.append(f"{tag}: sport {out['sport']} % 256 != {e['sport_mod256']}")
            if e.get("sport_lowport") and not (out["sport"] % 256 == 0 or out["sport"] == 1):
                errs.append(f"{tag}: sport {out['sport']} not a block's first port")
            if "same_ident" in e and out["ident"] != saved[e["same_ident"]][1]:
                errs.append(f"{tag}: identifier {out['ident']} != {saved[e['same_ident']][1]}")
            if "ident_next" in e and out["ident"] != saved[e["ident_next"]][1] + 1:
                errs.append(f"{tag}: identifier {out['ident']} != {saved[e['ident_next']][1]} + 1")
            if "src_net" in e and ipaddress.ip_address(out["src"]) not in ipaddress.ip_network(e["src_net"]):
                errs.append(f"{tag}: src {out['src']} outside {e['src_net']}")
            if "same" in e and (out["src"], out["sport"]) != saved[e["same"]][:2]:
                errs.append(f"{tag}: translation {(out['src'], out['sport'])} != {saved[e['same']][:2]}")
            for k in e.get("differs", ()):
                if (out["src"], out["sport"]) == saved[k][:2]:
                    errs.append(f"{tag}: translation {(out['src'], out['sport'])} reuses {k}'s")
        elif any(k in e for k in ("same", "differs", "src_net", "same_ident", "ident_next", "not_sport")):
            errs.append(f"{tag}: not delivered ({done})")
        if "flow" in e and (info is not None and info["ref"] != A.FLOW_NONE) != e["flow"]:
            errs.append(f"{tag}: flow attached {info is not None} != {e['flow']}")
        want = ("status", "not_status", "nat_status", "masq", "genid", "expires_in", "idle",
                "related_expires_in")
        fi = info if info is not None and info["ref"] != A.FLOW_NONE else None
        if fi is None and any(k in e for k in want):
            # a packet that created its flow pair carries none (the reference's
            # get_session looks it up): the forward flow by the packet's key
            fr = pkt.frame
            ks = np.zeros(1, A.FLOW_KEY)
            ks["src_vni"], ks["family"] = pkt.vni, 4
            ks["kind"] = {6: A.FLOW_TCP, 17: A.FLOW_UDP}.get(fr[23], A.FLOW_ICMP_QUERY)
            a, b = struct.unpack("!HH", fr[34:38])
            ks["sport"], ks["dport"] = (a, b) if fr[23] in (6, 17) else (struct.unpack("!H", fr[38:40])[0], 0)
            ks["src"][0, :4] = np.frombuffer(fr[26:30], np.uint8)
            ks["dst"][0, :4] = np.frombuffer(fr[30:34], np.uint8)
            got = r.lookup(ks)[0]
            fi = got if got["ref"] != A.FLOW_NONE else None
        if fi is not None:
            if "status" in e and fi["status"] != e["status"]:
                errs.append(f"{tag}: status {fi['status']} != {e['status']}")
            if "not_status" in e and fi["status"] == e["not_status"]:
                errs.append(f"{tag}: status {fi['status']} == {e['not_status']}")
            if "nat_status" in e and (fi["masq"] == A.PF_NONE or fi["pf_status"] != e["nat_status"]):
                errs.append(f"{tag}: nat status {fi['pf_status']} != {e['nat_status']}")
            if "masq" in e and fi["masq"] != e["masq"]:
                errs.append(f"{tag}: masquerade action {fi['masq']} != {e['masq']}")
            if "genid" in e and fi["genid"] != e["genid"]:
                errs.append(f"{tag}: genid {fi['genid']} != {e['genid']}")
            if "idle" in e and fi["idle_timeout_s"] != e["idle"]:
                errs.append(f"{tag}: idle timeout {fi['idle_timeout_s']} != {e['idle']}")
            if "expires_in" in e and int(fi["expires_at"]) < now + e["expires_in"]:
                errs.append(f"{tag}: expires_at {fi['expires_at']} < {now + e['expires_in']}")
            if "related_expires_in" in e:
                rel = r.get([int(fi["related"])])[0] if int(fi["related"]) != A.FLOW_NONE else None
                if rel is None or int(rel["expires_at"]) < now + e["related_expires_in"]:
                    errs.append(f"{tag}: related flow expiry too early")
        elif any(k in e for k in want):
            errs.append(f"{tag}: no flow")
        if "active" in e and r.count()[1] != e["active"]:
            errs.append(f"{tag}: active flows {r.count()[1]} != {e['active']}")
    return errs
