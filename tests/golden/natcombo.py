"""Known-answer tests of the NAT stages composed,
transcribed from the reference's own NAT pipeline tests (nat/src/test.rs).

The reference builds one pipeline -- IcmpErrorHandler, FlowLookup, the real
FlowFilter, StaticNat, PortForwarder, Masquerade (`setup_masq_pipeline`,
test.rs:69-139) -- from a validated overlay, and every table from that
overlay: the flow-filter context (`FlowFilterContext::try_from`), the static
NAT tables (`build_nat_configuration`), the port-forwarding table
(`update_from_vpc_table`) and the masquerade allocator
(`MasqueradeConfig::new`).  Here `lower()` restates those four lowerings for
the overlays of these tests, one packet is one burst through the whole path,
and an allocator update is a publish of the next generation:

- flow filter: `RuleSet::from_overlay` (flow-filter/src/context/tables.rs:
  566-676) -- per VPC and peering, stage 1 = the peer's public prefixes
  (masquerade ones gated on the peer VNI, port forwarding with the priority
  tie bit, `rule_priority` :452-454), stage 2 = the VPC's own private
  prefixes (port forwarding gated on PortFwdReply);
- static NAT: `PerVniTable::add_peering` over the static exposes only
  (nat/src/static_nat/setup/mod.rs:55-100; tests/golden/natcfg.py);
- port forwarding: `vpc_port_fw_peering` (nat/src/portfw/portfwtable/
  setup.rs:60-91): one rule per local port-forwarding expose, keyed on the
  remote VPC, TCP and UDP for a protocol-less expose;
- masquerade: one expose per local masquerade expose, the claims of the same
  manifest's port-forwarding exposes (nat/src/masquerade/apalloc/setup.rs:
  73-137).

Steps assert what the reference asserts (addresses, ports, DoneReason, the
flow count); the masquerade-allocated port is read from the output as the
reference test reads it.  The GPU runs every step against the oracle bit for
bit (tests/test_gpu_natcombo.py).
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from dataplane_amd import _abi as A
from dataplane_amd.tables import (NAT_MASQUERADE, NAT_NONE, NAT_PORT_FORWARDING, NAT_STATIC,
                                  TablesBuilder)
from golden import natcfg as N
from golden.kat import IF_MAC, NH_MAC, OIF_MAC, icmp4_err_frame
from golden.masqkat import REPLY, Pkt, Scenario, Step, l4_frame

TB = TablesBuilder
ANY = None
MODE = {"plain": NAT_NONE, "static": NAT_STATIC, "masq": NAT_MASQUERADE, "pf": NAT_PORT_FORWARDING,
        "default": NAT_NONE}


def pwp(prefix: str, lo: int, hi: int) -> Tuple[str, Tuple[int, int]]:
    """PrefixWithOptionalPorts with a port range (test.rs:43-45)."""
    return (prefix, (lo, hi))


def _pfx(p) -> Tuple[str, Optional[Tuple[int, int]]]:
    return (p, None) if isinstance(p, str) else p


@dataclass
class Exp:
    """A VpcExpose: `kind` plain / static (make_static_nat) / masq
    (make_masquerade) / pf (make_port_forwarding) / default (set_default: the
    catch-all, no prefixes); ips and as_range prefixes, each optionally with a
    port range; `proto` 6 / 17 or ANY."""
    kind: str
    ips: List
    as_range: List = field(default_factory=list)
    proto: Optional[int] = ANY
    idle_s: int = 0

    def public(self):
        return self.as_range if self.kind != "plain" else self.ips


@dataclass
class Peering:
    vni_a: int
    exposes_a: List[Exp]
    vni_b: int
    exposes_b: List[Exp]


def lower(peerings: List[Peering], genid: int = 1, randomize: bool = True,
          seed: int = 0x5EED) -> TablesBuilder:
    t = TB(genid=genid)
    t.masq_randomize, t.masq_seed = randomize, seed
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    vnis = sorted({v for p in peerings for v in (p.vni_a, p.vni_b)})
    for v in vnis:
        t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
    sides = []
    for p in peerings:
        sides.append((p.vni_a, p.exposes_a, p.vni_b, p.exposes_b))
        sides.append((p.vni_b, p.exposes_b, p.vni_a, p.exposes_a))
    static = []
    for (lv, local, rv, remote) in sides:
        # a default expose is the root prefix of the peering's version
        v6 = any(":" in _pfx(x)[0] for e in local + remote for x in e.ips + e.as_range)
        root = "::/0" if v6 else "0.0.0.0/0"
        # flow filter, stage 1: the peer's public prefixes
        for e in remote:
            if e.kind == "default":
                t.add_ff_remote(lv, root, rv, NAT_NONE)
                continue
            gate = rv if e.kind == "masq" else 0
            for pfx in e.public():
                pref, ports = _pfx(pfx)
                t.add_ff_remote(lv, pref, rv, MODE[e.kind], proto=e.proto,
                                dports=ports or (0, 65535), gate_vni=gate,
                                port_forwarding=e.kind == "pf")
        # stage 2: the VPC's own private prefixes
        for e in local:
            if e.kind == "default":
                t.add_ff_local(lv, rv, root, NAT_NONE)
                continue
            for pfx in e.ips:
                pref, ports = _pfx(pfx)
                t.add_ff_local(lv, rv, pref, MODE[e.kind], proto=e.proto,
                               sports=ports or (0, 65535), gate=1 if e.kind == "pf" else 0)
        # port forwarding: the local exposes, keyed on the remote VPC
        for e in local:
            if e.kind != "pf":
                continue
            (ip, iports), (ext, eports) = _pfx(e.ips[0]), _pfx(e.as_range[0])
            for proto in ((6, 17) if e.proto is ANY else (e.proto,)):
                t.add_portfw(src_vni=rv, proto=proto, dst_vni=lv, ext_prefix=ext, int_prefix=ip,
                             ext_ports=eports, int_ports=iports, estab_timeout_s=e.idle_s)
        # masquerade: the claims of the same manifest's port-forwarding exposes
        claims = []
        for e in local:
            if e.kind == "pf":
                pref, ports = _pfx(e.as_range[0])
                protos = {6: A.MASQ_TCP, 17: A.MASQ_UDP}.get(e.proto, A.MASQ_TCP | A.MASQ_UDP)
                claims.append((pref, ports[0], ports[1], protos))
        for e in local:
            if e.kind == "masq":
                t.add_masquerade(lv, rv, [_pfx(x)[0] for x in e.ips],
                                 [_pfx(x)[0] for x in e.as_range], idle_timeout_s=e.idle_s,
                                 claims=claims)
        static.append(N.Peering(lv, rv,
                                [N.Expose(ips=list(e.ips), as_range=list(e.as_range))
                                 for e in local if e.kind == "static"],
                                [N.Expose(ips=list(e.ips), as_range=list(e.as_range))
                                 for e in remote if e.kind == "static"]))
    N.lower(t, N.nat_tables(static))
    return t


# ---------------------------------------------------------------------------
# the overlays of nat/src/test.rs
# ---------------------------------------------------------------------------
V1, V2 = 100, 200


def overlapping_masquerade_and_port_forward() -> List[Peering]:
    """build_overlapping_masquerade_and_port_forward (test.rs:141-174): the
    internal VPC masquerades 192.168.0.0/24 behind 5.6.7.8 and forwards
    5.6.7.8:1024 to 192.168.0.8:8000 -- the same public address."""
    return [Peering(V1, [Exp("plain", ["1.2.3.0/24"])],
                    V2, [Exp("masq", ["192.168.0.0/24"], ["5.6.7.8/32"]),
                         Exp("pf", [pwp("192.168.0.8/32", 8000, 8000)],
                             [pwp("5.6.7.8/32", 1024, 1024)])])]


def static_masquerade() -> List[Peering]:
    """test_nat_combination_static_masquerade (test.rs:251-357) and its ICMP
    error variant (:482-608)."""
    return [Peering(V1, [Exp("masq", ["1.2.3.0/24"], ["5.5.5.5/32"])],
                    V2, [Exp("static", ["192.168.0.0/24"], ["5.6.7.0/24"])])]


def static_portfw() -> List[Peering]:
    """test_nat_combination_static_portfw (test.rs:358-480): static PAT on
    one side, port forwarding on the other."""
    return [Peering(V1, [Exp("static", [pwp("1.2.3.0/24", 1201, 1300)],
                             [pwp("5.5.5.0/24", 1701, 1800)])],
                    V2, [Exp("pf", [pwp("192.168.0.0/24", 7001, 8000)],
                             [pwp("5.6.7.0/24", 5001, 6000)])])]


def static_portfw_icmp() -> List[Peering]:
    """test_nat_combination_static_portfwd_icmp_error (test.rs:609-739):
    address-only static NAT on one side, port forwarding on the other."""
    return [Peering(V1, [Exp("static", ["1.2.3.0/24"], ["5.5.5.0/24"])],
                    V2, [Exp("pf", [pwp("192.168.0.0/24", 7001, 8000)],
                             [pwp("5.6.7.0/24", 5001, 6000)])])]


OVERLAYS = {
    "overlap": overlapping_masquerade_and_port_forward,
    "static_masq": static_masquerade,
    "static_portfw": static_portfw,
    "static_portfw_icmp": static_portfw_icmp,
}


def builder(randomize_by_gen: Optional[Dict[int, bool]] = None):
    """(overlay, genid) -> TablesBuilder; `randomize_by_gen`: the allocator's
    set_randomize per generation (the reference's default: true)."""
    def mk(name: str, genid: int) -> TablesBuilder:
        rnd = True if randomize_by_gen is None else randomize_by_gen.get(genid, True)
        return lower(OVERLAYS[name](), genid, randomize=rnd)
    return mk


def udp(src: str, dst: str, sport: int, dport: int, vni: int) -> Pkt:
    """build_packet (test.rs:47-67): UDP over IPv4, overlay, src VPC set."""
    return Pkt(l4_frame(src, dst, 17, sport, dport), vni)


def icmp_err_for(saved: str, router: str = "9.10.11.12", vni: int = V2):
    """build_test_icmp4_destination_unreachable_packet(router, src of the
    saved output, that output's src / dst, UDP, its ports) from VPC `vni`."""
    def mk(sv, _last):
        o = sv[saved][2][0]
        return Pkt(icmp4_err_frame(router, o["src"], o["src"], o["dst"], 17, o["sport"], o["dport"]),
                   vni)
    return mk


def reply_to(saved: str, vni: int):
    """The reply of a saved output: addresses and ports swapped, from `vni`."""
    def mk(sv, _last):
        o = sv[saved][2][0]
        return udp(o["dst"], o["src"], o["dport"], o["sport"], vni)
    return mk


def scenarios() -> List[Scenario]:
    t = "nat/src/test.rs"
    sc = []
    # a_port_forwarded_tuple_is_never_masqueraded (:176-199), set_randomize(false)
    sc.append(Scenario("port_forwarded_tuple_never_masqueraded", f"{t}:176-199", "overlap", [
        Step(udp("192.168.0.9", "1.2.3.10", 4000, 9000, V2),
             dict(done="Delivered", src="5.6.7.8", not_sport=1024)),
    ], build=builder({1: False, 2: False})))
    # a_claimed_tuple_cannot_be_reserved_for_masquerade (:201-247): two clients
    # reach the forwarded service through the claimed tuple; the claim holds
    # (reserve_port Denied, seen here as masquerade never handing the tuple
    # out: the deterministic allocator's first port would be 1024) and
    # survives an allocator replacement (generation 3, randomized)
    claim = [Step(udp(c, "5.6.7.8", p, 1024, V1),
                  dict(done="Delivered", dst="192.168.0.8", dport=8000))
             for (c, p) in (("1.2.3.4", 5000), ("1.2.3.5", 5001))]
    masq = [Step(udp("192.168.0.9", "1.2.3.10", 4000 + k, 9000, V2),
                 dict(done="Delivered", src="5.6.7.8", not_sport=1024)) for k in range(8)]
    sc.append(Scenario("claimed_tuple_cannot_be_reserved_for_masquerade", f"{t}:201-247", "overlap",
                       claim + masq + [
        Step(udp("1.2.3.4", "5.6.7.8", 5000, 1024, V1),
             dict(done="Delivered", dst="192.168.0.8", dport=8000), publish=("overlap", 3)),
        Step(udp("1.2.3.6", "5.6.7.8", 5002, 1024, V1),
             dict(done="Delivered", dst="192.168.0.8", dport=8000)),
    ] + [Step(udp("192.168.0.9", "1.2.3.10", 5000 + k, 9000, V2),
              dict(done="Delivered", src="5.6.7.8", not_sport=1024)) for k in range(8)],
        build=builder({1: False, 2: False, 3: True})))
    # test_nat_combination_static_masquerade (:249-356)
    sc.append(Scenario("static_masquerade", f"{t}:249-356", "static_masq", [
        Step(udp("1.2.3.4", "5.6.7.8", 1234, 5678, V1),
             dict(done="Delivered", src="5.5.5.5", dst="192.168.0.8", dport=5678), save="out"),
        Step(reply_to("out", V2), dict(done="Delivered", src="5.6.7.8", dst="1.2.3.4", sport=5678,
                                       dport=1234)),
        Step(udp("1.2.3.4", "5.6.7.8", 1234, 5678, V1),
             dict(done="Delivered", src="5.5.5.5", dst="192.168.0.8", same="out")),
        Step(None, dict(flows=2)),
    ], build=builder()))
    # test_nat_combination_static_portfw (:358-480)
    sc.append(Scenario("static_portfw", f"{t}:358-480", "static_portfw", [
        Step(udp("1.2.3.4", "5.6.7.8", 1234, 5678, V1),
             dict(done="Delivered", src="5.5.5.4", dst="192.168.0.8", sport=1734, dport=7678)),
        Step(udp("192.168.0.8", "5.5.5.4", 7678, 1734, V2),
             dict(done="Delivered", src="5.6.7.8", dst="1.2.3.4", sport=5678, dport=1234)),
        Step(None, dict(flows=2)),
        Step(udp("1.2.3.4", "5.6.7.8", 1234, 5678, V1),
             dict(done="Delivered", src="5.5.5.4", dst="192.168.0.8")),
    ], build=builder()))
    # test_nat_combination_static_masq_icmp_error (:482-607): the outer
    # destination and the embedded packet translated back
    sc.append(Scenario("static_masq_icmp_error", f"{t}:482-607", "static_masq", [
        Step(udp("1.2.3.4", "5.6.7.8", 1234, 5678, V1),
             dict(done="Delivered", src="5.5.5.5", dst="192.168.0.8"), save="out"),
        Step(icmp_err_for("out"), dict(done="Delivered", src="9.10.11.12", dst="1.2.3.4",
                                       isrc="1.2.3.4", idst="5.6.7.8", isport=1234, idport=5678)),
    ], build=builder()))
    # test_nat_combination_static_portfwd_icmp_error (:609-739): the outer
    # source becomes the original destination
    sc.append(Scenario("static_portfwd_icmp_error", f"{t}:609-739", "static_portfw_icmp", [
        Step(udp("1.2.3.4", "5.6.7.8", 1234, 5678, V1),
             dict(done="Delivered", src="5.5.5.4", dst="192.168.0.8", sport=1234, dport=7678),
             save="out"),
        Step(icmp_err_for("out"), dict(done="Delivered", src="5.6.7.8", dst="1.2.3.4",
                                       isrc="1.2.3.4", idst="5.6.7.8", isport=1234, idport=5678)),
    ], build=builder()))
    return sc
