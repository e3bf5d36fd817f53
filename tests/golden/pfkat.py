"""Known-answer tests of port forwarding, transcribed
from the reference's own PortForwarder tests (nat/src/portfw/test.rs:221-801).

The reference tests run FlowLookup -> a test flow filter (which only sets the
destination VPC) -> PortForwarder, packet by packet, with the
port-forwarding table updated by hand in between.  Here each packet is a
burst of its own through the whole path, with flow-filter tables that route
vpc1 (VNI 2000) to vpc2 (VNI 3000) through a port-forwarding expose (the
remote rule of 70.71.72.0/24 carries NatRequirement::PortForwarding, so the
flow filter sets the port-forwarding requirement the reference tests set by
hand); replies are forwarded on their flows (the flow filter's bypass).  A
rule-set change is a publish of the same generation, as the reference test
updates only the PortFwTable.  The flow clock (DP_OPT_CLOCK) stands for
Instant::now(); the flow timers are dp_flow_sweep.

Each scenario step checks what the reference test asserts: DoneReason, the
translated addresses and ports, the packet's flow (FlowStatus, NatFlowStatus,
expiry, whether its rule's Weak still upgrades) and the flow count.
"""
from __future__ import annotations

import ipaddress
import struct
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.tables import NAT_NONE, NAT_PORT_FORWARDING, TablesBuilder
from edgecase import pack_burst
from golden.kat import IF_MAC, NH_MAC, OIF_MAC, PEER_MAC
import pktgen as P

TB = TablesBuilder
VPC1, VPC2, VPC3 = 2000, 3000, 4000
SEC = 1_000_000_000
FIN, SYN, RST, PSH, ACK = 0x01, 0x02, 0x04, 0x08, 0x10


def frame(src: str, dst: str, proto: int, sport: int, dport: int, flags: int = 0) -> bytes:
    """build_test_{tcp,udp}_ipv4_packet (net/src/packet/test_utils.rs:178-226):
    the TCP header's flags all clear unless set."""
    if proto == 6:
        body = P.tcp(sport, dport, b"", P.pseudo4(src, dst, 6, 20), flags=flags)
    else:
        body = P.udp(sport, dport, b"", P.pseudo4(src, dst, 17, 8))
    return P.eth(IF_MAC, PEER_MAC, 0x0800) + P.ipv4(src, dst, proto, len(body)) + body


def fields(fr: bytes) -> dict:
    """src / dst address and ports (and TCP flags) of a serialized IPv4 frame."""
    ihl = (fr[14] & 15) * 4
    l4 = 14 + ihl
    sp, dp = struct.unpack("!HH", fr[l4:l4 + 4])
    return dict(src=str(ipaddress.ip_address(fr[26:30])), dst=str(ipaddress.ip_address(fr[30:34])),
                sport=sp, dport=dp, proto=fr[23], flags=fr[l4 + 13] if fr[23] == 6 else 0)


def reply_of(out: dict, vni: int) -> "Pkt":
    """build_reply (test.rs:69-97): addresses and ports swapped, from the
    packet's destination VPC; TCP: SYN|ACK loses SYN, ACK is set."""
    fl = out["flags"]
    if out["proto"] == 6:
        if fl & SYN and fl & ACK:
            fl &= ~SYN
        fl |= ACK
    return Pkt(frame(out["dst"], out["src"], out["proto"], out["dport"], out["sport"], fl), vni)


def world(rules: List[dict], genid: int = 1) -> Callable[[], TablesBuilder]:
    """vpc1 -> vpc2 through a port-forwarding expose of 70.71.72.0/24 (any
    protocol), clients in 10.0.0.0/8; every VPC routes 0/0 to a resolved
    next hop.  rules: add_portfw kwargs."""
    def build():
        t = TB(genid=genid)
        t.add_iface(1, IF_MAC)
        t.add_iface(10, OIF_MAC)
        t.add_adjacency("192.0.2.1", 10, NH_MAC)
        nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
        t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
        for v in (VPC1, VPC2, VPC3):
            t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
        t.add_ff_remote(VPC1, "70.71.72.0/24", VPC2, NAT_PORT_FORWARDING, port_forwarding=True)
        t.add_ff_local(VPC1, VPC2, "10.0.0.0/8")
        # vpc2's side: the port-forwarded hosts, gated on PortFwdReply (only a
        # reply flow's revalidation reaches them, flow-filter/src/context/tables.rs:624-648)
        t.add_ff_remote(VPC2, "10.0.0.0/8", VPC1)
        t.add_ff_local(VPC2, VPC1, "192.168.0.0/16", NAT_PORT_FORWARDING, gate=1)
        for r in rules:
            t.add_portfw(**r)
        return t
    return build


def tcp_rule(ext="70.71.72.73/32", intl="192.168.1.1/32", ext_ports=(3022, 3022),
             int_ports=(22, 22), dst=VPC2, **kw):
    return dict(src_vni=VPC1, proto=6, dst_vni=dst, ext_prefix=ext, int_prefix=intl,
                ext_ports=ext_ports, int_ports=int_ports, **kw)


def udp_rule(ext="70.71.72.73/32", intl="192.168.1.2/32", ext_ports=(3053, 3053),
             int_ports=(53, 53), dst=VPC2, **kw):
    return dict(src_vni=VPC1, proto=17, dst_vni=dst, ext_prefix=ext, int_prefix=intl,
                ext_ports=ext_ports, int_ports=int_ports, **kw)


def base_rules():  # build_test_port_forwarding_ruleset (test.rs:99-130)
    return [tcp_rule(), udp_rule()]


@dataclass
class Pkt:
    frame: bytes
    vni: int


def udp_fwd() -> Pkt:  # udp_packet_to_port_forward (test.rs:132-140)
    return Pkt(frame("10.0.0.1", "70.71.72.73", 17, 9876, 3053), VPC1)


def tcp_fwd(flags=0) -> Pkt:  # tcp_packet_to_port_forward (test.rs:142-154)
    return Pkt(frame("10.0.0.2", "70.71.72.73", 6, 7777, 3022, flags), VPC1)


def tcp_rev(flags=0, src="192.168.1.1", sport=22) -> Pkt:  # tcp_packet_reverse_reply (:156-167)
    return Pkt(frame(src, "10.0.0.2", 6, sport, 7777, flags), VPC2)


REPLY = "reply"   # a step whose packet is the reply of the previous step's output


@dataclass
class Step:
    pkt: object                        # Pkt, or REPLY
    expect: Dict = field(default_factory=dict)
    publish: Optional[List[dict]] = None   # publish these rules (same generation) first
    sweep: bool = False                # fire the flow timers up to the clock first
    advance: int = SEC                 # the clock moves this much before the step


@dataclass
class Scenario:
    name: str
    ref: str
    rules: List[dict]
    steps: List[Step]


def establish() -> List[Step]:  # establish_tcp_connection (test.rs:294-319)
    return [Step(tcp_fwd(SYN), dict(done="Delivered")),
            Step(REPLY, dict(flow=True, status=A.FLOW_ACTIVE, pf_status=A.NFS_TWO_WAY)),
            Step(tcp_fwd(ACK), dict(done="Delivered", status=A.FLOW_ACTIVE,
                                    pf_status=A.NFS_ESTABLISHED))]


def scenarios() -> List[Scenario]:
    t = "nat/src/portfw/test.rs"
    sc = []
    sc.append(Scenario("base", f"{t}:221-271", base_rules(), [
        Step(udp_fwd(), dict(done="Delivered", src="10.0.0.1", dst="192.168.1.2", sport=9876,
                             dport=53, flow=False)),
        Step(REPLY, dict(done="Delivered", src="70.71.72.73", dst="10.0.0.1", sport=3053,
                         dport=9876, status=A.FLOW_ACTIVE, pf_status=A.NFS_TWO_WAY,
                         expires_in=10 * SEC)),
        Step(udp_fwd(), dict(done="Delivered", src="10.0.0.1", dst="192.168.1.2", sport=9876,
                             dport=53, status=A.FLOW_ACTIVE, expires_in=30 * SEC)),
    ]))
    sc.append(Scenario("tcp_filtered", f"{t}:273-292", base_rules(), [
        Step(tcp_fwd(), dict(done="NatNotPortForwarded")),
        Step(tcp_rev(), dict(flow=False)),
    ]))
    sc.append(Scenario("tcp_establishment", f"{t}:321-331", base_rules(), establish()))
    sc.append(Scenario("tcp_close_server", f"{t}:333-369", base_rules(), establish() + [
        Step(tcp_rev(FIN), dict(flow=True, status=A.FLOW_ACTIVE, pf_status=A.NFS_S_CLOSING)),
        Step(tcp_fwd(ACK | FIN), dict(done="Delivered", status=A.FLOW_ACTIVE,
                                      pf_status=A.NFS_LAST_ACK)),
        Step(tcp_rev(ACK), dict(flow=True, not_status=A.FLOW_ACTIVE, pf_status=A.NFS_CLOSED,
                                flows=2)),
    ]))
    sc.append(Scenario("tcp_close_client", f"{t}:371-405", base_rules(), establish() + [
        Step(tcp_fwd(FIN), dict(flow=True, pf_status=A.NFS_C_CLOSING)),
        Step(tcp_rev(ACK | FIN), dict(done="Delivered", pf_status=A.NFS_LAST_ACK)),
        Step(tcp_rev(ACK), dict(flow=True, not_status=A.FLOW_ACTIVE, pf_status=A.NFS_CLOSED,
                                flows=2)),
    ]))
    sc.append(Scenario("tcp_half_close_client", f"{t}:407-451", base_rules(), establish() + [
        Step(tcp_fwd(FIN), dict(flow=True, pf_status=A.NFS_C_CLOSING)),
        Step(tcp_rev(ACK), dict(done="Delivered", pf_status=A.NFS_C_HALF_CLOSE)),
        Step(tcp_rev(FIN), dict(flow=True, pf_status=A.NFS_LAST_ACK)),
        Step(tcp_fwd(ACK), dict(flow=True, not_status=A.FLOW_ACTIVE, pf_status=A.NFS_CLOSED,
                                flows=2)),
    ]))
    sc.append(Scenario("tcp_reset", f"{t}:453-488", base_rules(), [
        Step(tcp_fwd(SYN)),
        Step(REPLY),
        Step(tcp_fwd(ACK), dict(pf_status=A.NFS_ESTABLISHED)),
        Step(tcp_fwd(RST), dict(done="Delivered", status=A.FLOW_CANCELLED,
                                pf_status=A.NFS_RESET, flows=2)),
    ]))
    sc.append(Scenario("config_removal_interrupts_traffic", f"{t}:490-541", base_rules(), [
        Step(tcp_fwd(SYN), dict(done="Delivered")),
        Step(tcp_rev(SYN | ACK), dict(flow=True, pf_status=A.NFS_TWO_WAY)),
        Step(tcp_fwd(ACK), dict(done="Delivered", pf_status=A.NFS_ESTABLISHED)),
        Step(tcp_fwd(), dict(done="NatNotPortForwarded"), publish=base_rules()[1:]),
        Step(tcp_fwd(), dict(done="NatNotPortForwarded", flow=False), sweep=True,
             advance=4 * SEC),
    ]))
    ranges = [udp_rule(ext_ports=(3000, 3100), int_ports=(2000, 2100))]
    sc.append(Scenario("with_port_ranges", f"{t}:612-651", ranges, [
        Step(udp_fwd(), dict(done="Delivered", dst="192.168.1.2", dport=2053)),
        Step(udp_fwd(), dict(rule_alive=True, flows=2)),
        Step(REPLY, dict(done="Delivered", rule_alive=True)),
        Step(udp_fwd(), dict(rule_alive=False, flows=2), publish=[]),
    ]))
    pfx = [udp_rule(ext="70.71.72.70/24", intl="192.168.6.0/24", ext_ports=(3000, 3100),
                    int_ports=(2000, 2100))]
    sc.append(Scenario("with_prefixes_and_port_ranges", f"{t}:653-692", pfx, [
        Step(udp_fwd(), dict(done="Delivered", dst="192.168.6.73", dport=2053)),
        Step(udp_fwd(), dict(rule_alive=True, flows=2)),
        Step(REPLY, dict(done="Delivered", rule_alive=True)),
        Step(udp_fwd(), dict(rule_alive=False, flows=2), publish=[]),
    ]))
    wide = [tcp_rule(ext="70.71.72.0/24", intl="192.168.1.0/24", ext_ports=(3010, 3050),
                     int_ports=(10, 50))]
    narrow = [tcp_rule(ext="70.71.72.73/32", intl="192.168.1.73/32", ext_ports=(3022, 3023),
                       int_ports=(22, 23))]
    sc.append(Scenario("compatible_rule_updates_preserve_flows", f"{t}:694-746", wide,
                       establish() + [
        Step(tcp_fwd(), dict(flow=True, status=A.FLOW_ACTIVE, pf_status=A.NFS_ESTABLISHED,
                             rule="new", flows=2), publish=narrow),
    ]))
    moved = [tcp_rule(ext="70.71.72.0/24", intl="192.168.2.0/24", ext_ports=(3010, 3050),
                      int_ports=(10, 50))]
    sc.append(Scenario("incompatible_rule_updates_remove_flows", f"{t}:748-801", wide,
                       establish() + [
        Step(tcp_fwd(), dict(flow=True, status=A.FLOW_CANCELLED, pf_status=A.NFS_ESTABLISHED,
                             rule_alive=False, done="NatNotPortForwarded"), publish=moved),
    ]))
    return sc


# ---------------------------------------------------------------------------
# runners
# ---------------------------------------------------------------------------
class OracleRunner:
    """The oracle (CPU restatement) as one device: tables generation lineage,
    a flow table and the flow clock."""

    def __init__(self, **_):
        from oracle.pyoracle import Oracle, OracleFlows
        self._Oracle = Oracle
        self.fl = OracleFlows()
        self.tabs = None
        self.keep = []

    def publish(self, builder: TablesBuilder):
        self.keep.append(builder)
        self.tabs = self._Oracle(builder.build(), prev=self.tabs)

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

    def rule_alive(self, rule_id):
        return self.tabs.rule_alive(rule_id)

    def live_rules(self):
        return None


class GpuRunner:
    """The HIP path through the C ABI: one context, its flow table."""

    def __init__(self, slots: int = 1 << 12):
        from dataplane_amd import GpuPathNf
        from dataplane_amd.flows import FlowTable
        self.nf = GpuPathNf(0)
        self.ft = FlowTable(0, slots)
        self.nf.attach_flows(self.ft)
        self.keep = []

    def publish(self, builder: TablesBuilder):
        self.keep.append(builder)
        self.nf.publish(builder.build())

    def set_clock(self, ns: int):
        self.nf.set_option(A.OPT_CLOCK, ns)

    def burst(self, buf, inp):
        return self.nf.process_arrays(buf, inp)

    def get(self, refs):
        return self.ft.get(np.asarray(refs, np.uint64))

    def count(self):
        return self.ft.count()

    def sweep(self, now):
        return self.ft.sweep(now)

    def lookup(self, keys):
        return self.ft.lookup(keys)

    def nat_counters(self):
        """The last burst's NAT-pass counters (dp_flow.h FlowCtx::pf_cnt):
        [12] the mode that ran (1 one lane, 2 connections, 3 split), [11]
        records on the allocating lane, [13] left there by connection lanes,
        [14] allocations in wave batches, [15] alone, [16] pairs refused."""
        import ctypes as C
        out = (C.c_uint32 * 40)()
        n = A.gpu_lib().dpf_debug_nat_counters(self.nf.ctx, out, 40)
        assert n == 40, n
        return np.array(out[:], dtype=np.uint32)

    def close(self):
        self.nf.attach_flows(None)
        self.nf.close()
        self.ft.close()


def run_scenario(s: Scenario, r, on_step=None) -> List[str]:
    """Run one scenario on runner `r`; returns the failed expectations.
    on_step(i, res, buf, infos) sees every step's records, buffer and the
    packet's flow info (for cross-runner comparison)."""
    errs: List[str] = []
    now = 0
    rules = s.rules
    r.publish(world(rules)())
    prev_out = None
    rule_ids = {}
    for i, st in enumerate(s.steps):
        now += st.advance
        r.set_clock(now)
        if st.publish is not None:
            rules = st.publish
            r.publish(world(rules)())
        if st.sweep:
            r.sweep(now)
        pkt = st.pkt
        if pkt == REPLY:
            pkt = reply_of(prev_out, VPC2 if prev_out["dst"].startswith("192.168.") else VPC1)
        buf, inp = pack_burst([(pkt.frame, 1, A.IN_SEEDED_OVERLAY, pkt.vni)])
        res = r.burst(buf, inp)
        o = res[0]
        done = A.DONE_NAMES[o["done"]] if o["done"] < A.DONE_COUNT else str(o["done"])
        out = None
        if done == "Delivered":
            out = fields(buf[o["off"]:o["off"] + o["len"]].tobytes())
            prev_out = out
        ref = int(o["flow_ref"])
        info = r.get([ref])[0] if ref != A.FLOW_NONE else None
        if on_step:
            on_step(i, res, buf, info)
        e = st.expect
        tag = f"{s.name} step {i}"
        if "done" in e and done != e["done"]:
            errs.append(f"{tag}: done {done} != {e['done']}")
        for k in ("src", "dst", "sport", "dport"):
            if k in e and (out is None or out[k] != e[k]):
                errs.append(f"{tag}: {k} {None if out is None else out[k]} != {e[k]}")
        if "flow" in e and (info is not None and info["ref"] != A.FLOW_NONE) != e["flow"]:
            errs.append(f"{tag}: flow attached {info is not None} != {e['flow']}")
        if info is not None:
            if "status" in e and info["status"] != e["status"]:
                errs.append(f"{tag}: status {info['status']} != {e['status']}")
            if "not_status" in e and info["status"] == e["not_status"]:
                errs.append(f"{tag}: status {info['status']} == {e['not_status']}")
            if "pf_status" in e and info["pf_status"] != e["pf_status"]:
                errs.append(f"{tag}: pf_status {info['pf_status']} != {e['pf_status']}")
            if "expires_in" in e and int(info["expires_at"]) < now + e["expires_in"]:
                errs.append(f"{tag}: expires_at {info['expires_at']} < {now + e['expires_in']}")
            if "rule_alive" in e and hasattr(r, "rule_alive"):
                if r.rule_alive(int(info["pf_rule"])) != e["rule_alive"]:
                    errs.append(f"{tag}: rule alive != {e['rule_alive']}")
            if e.get("rule") == "new":
                # the flow now names the entry of the new rule set (the only one)
                if hasattr(r, "rule_alive") and not r.rule_alive(int(info["pf_rule"])):
                    errs.append(f"{tag}: flow's rule is not the new entry")
                rule_ids["new"] = int(info["pf_rule"])
        elif any(k in e for k in ("status", "pf_status", "rule_alive")):
            errs.append(f"{tag}: no flow attached")
        if "flows" in e and r.count()[0] != e["flows"]:
            errs.append(f"{tag}: flow table len {r.count()[0]} != {e['flows']}")
    return errs
