"""Seeded port-forwarding workload for bench.py's NAT leg (harness, not the
product path): a burst in which a chosen share of the packets opens a new
port-forwarded connection and the rest is plain routed traffic.

World: VPC 100's clients (10.0.0.0/8) reach VPC 200's servers through one
port-forwarding rule, external 70.71.0.0/16 UDP ports 3000-3999 onto internal
192.168.0.0/16 ports 5000-5999 (PortFwEntry, nat/src/portfw/portfwtable/
objects.rs:70-103); VPC 100 also routes 172.16.0.0/12 to VPC 300 without NAT
(the plain share).  Every packet is a 64-byte Ethernet / IPv4 / UDP frame from
a distinct client address and port, so each port-forwarded packet creates its
own flow pair (PortForwarder's try_port_forwarding, nat/src/portfw/nf.rs:
174-204)."""
from __future__ import annotations

import numpy as np

from . import _abi as A
from .tables import NAT_MASQUERADE, NAT_PORT_FORWARDING, TablesBuilder as TB

VPC_C, VPC_S, VPC_P = 100, 200, 300
IF_MAC, OIF_MAC, PEER_MAC, NH_MAC = ("02:00:00:00:00:01", "02:00:00:00:00:0a",
                                     "02:00:00:00:00:99", "02:00:00:00:00:42")
FRAME = 64
SLOT = 192  # headroom + frame, 64-byte aligned (DPDK-like)


def tables(genid: int = 1) -> TB:
    t = TB(genid=genid)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    for v in (VPC_C, VPC_S, VPC_P):
        t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
    t.add_ff_remote(VPC_C, "70.71.0.0/16", VPC_S, NAT_PORT_FORWARDING, port_forwarding=True)
    t.add_ff_local(VPC_C, VPC_S, "10.0.0.0/8")
    t.add_ff_remote(VPC_C, "172.16.0.0/12", VPC_P)
    t.add_ff_local(VPC_C, VPC_P, "10.0.0.0/8")
    t.add_ff_remote(VPC_S, "10.0.0.0/8", VPC_C)
    t.add_ff_local(VPC_S, VPC_C, "192.168.0.0/16", NAT_PORT_FORWARDING, gate=1)
    t.add_portfw(src_vni=VPC_C, proto=17, dst_vni=VPC_S, ext_prefix="70.71.0.0/16",
                 int_prefix="192.168.0.0/16", ext_ports=(3000, 3999), int_ports=(5000, 5999))
    return t


def masq_tables(genid: int = 1) -> TB:
    """The masquerade world: VPC 100's clients (10.0.0.0/8) reach VPC 200's
    198.18.0.0/15 masqueraded behind the public pool 203.0.113.0/24 (256
    addresses, 64512 ports each: MasqueradeConfig, nat/src/masquerade/
    allocator_writer.rs:43-61, deterministic allocator), lowered as the
    reference's flow-filter tables lower a masquerading peering (remote
    rules, ungated and gated on the peer; a local rule requiring masquerade);
    172.16.0.0/12 routes to VPC 300 without NAT (the plain share)."""
    t = TB(genid=genid)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    for v in (VPC_C, VPC_S, VPC_P):
        t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
    t.add_masquerade(VPC_C, VPC_S, ["10.0.0.0/8"], ["203.0.113.0/24"])
    t.add_ff_remote(VPC_C, "198.18.0.0/15", VPC_S)
    t.add_ff_remote(VPC_C, "198.18.0.0/15", VPC_S, gate_vni=VPC_S)
    t.add_ff_local(VPC_C, VPC_S, "10.0.0.0/8", NAT_MASQUERADE)
    t.add_ff_remote(VPC_C, "172.16.0.0/12", VPC_P)
    t.add_ff_local(VPC_C, VPC_P, "10.0.0.0/8")
    return t


def _ip(a: np.ndarray) -> np.ndarray:
    """u32 addresses -> (n, 4) big-endian bytes"""
    return a.astype(">u4").view(np.uint8).reshape(-1, 4)


def burst(n: int, pf_share: float, step: int, seed: int = 1, kind: str = "pf"):
    """(buf, inp): n frames in SLOT-byte slots, the first bytes of each slot
    headroom; packet i opens a new stateful-NAT connection with probability
    pf_share -- port-forwarded (kind "pf": 70.71.0.0/16 UDP 3000-3999) or
    masqueraded (kind "masq": 198.18.0.0/15, any port; masq_tables).  `step`
    moves the clients, so every step's connections are new."""
    rng = np.random.default_rng(seed * 1000 + step)
    pf = rng.random(n) < pf_share
    idx = np.arange(n, dtype=np.uint64)
    # distinct clients: 10.<step>.x.y, one port each
    src = (np.uint64(10 << 24) + np.uint64((step & 0xff) << 16) + (idx >> np.uint64(6))).astype(np.uint32)
    sport = (1024 + (idx & np.uint64(63)) * 900 + np.uint64(step % 900)).astype(np.uint16)
    if kind == "masq":
        dst_pf = (np.uint32(198 << 24 | 18 << 16) + rng.integers(1, 1 << 17, n).astype(np.uint32))
        dport_pf = rng.integers(1, 65535, n)
    else:
        dst_pf = (np.uint32(70 << 24 | 71 << 16) + rng.integers(1, 65535, n).astype(np.uint32))
        dport_pf = rng.integers(3000, 4000, n)
    dst_pl = (np.uint32(172 << 24 | 16 << 16) + rng.integers(1, 1 << 20, n).astype(np.uint32))
    dst = np.where(pf, dst_pf, dst_pl).astype(np.uint32)
    dport = np.where(pf, dport_pf, rng.integers(1, 65535, n)).astype(np.uint16)
    fr = np.zeros((n, FRAME), dtype=np.uint8)
    mac = lambda s: np.frombuffer(bytes(int(x, 16) for x in s.split(":")), np.uint8)
    fr[:, 0:6] = mac(IF_MAC)
    fr[:, 6:12] = mac(PEER_MAC)
    fr[:, 12:14] = (0x08, 0x00)
    ip = fr[:, 14:34]
    ip[:, 0] = 0x45
    ip[:, 2:4] = np.array([0, FRAME - 14], np.uint8)
    ip[:, 8] = 64
    ip[:, 9] = 17
    ip[:, 12:16] = _ip(src)
    ip[:, 16:20] = _ip(dst)
    words = ip.reshape(n, 10, 2).astype(np.uint32)
    s = (words[:, :, 0] << 8 | words[:, :, 1]).sum(axis=1)
    s = (s & 0xffff) + (s >> 16)
    s = (s & 0xffff) + (s >> 16)
    ck = (~s & 0xffff).astype(np.uint16)
    ip[:, 10] = ck >> 8
    ip[:, 11] = ck & 0xff
    udp = fr[:, 34:42]
    udp[:, 0:2] = sport.astype(">u2").view(np.uint8).reshape(-1, 2)
    udp[:, 2:4] = dport.astype(">u2").view(np.uint8).reshape(-1, 2)
    udp[:, 4:6] = np.array([0, FRAME - 34], np.uint8)  # checksum 0: none (IPv4)
    head = SLOT - FRAME
    buf = np.zeros(n * SLOT + 64, dtype=np.uint8)
    buf[: n * SLOT].reshape(n, SLOT)[:, head:] = fr
    inp = np.zeros(n, dtype=A.PKT_IN)
    inp["off"] = np.arange(n, dtype=np.uint32) * SLOT + head
    inp["len"] = FRAME
    inp["flags"] = A.IN_SEEDED_OVERLAY
    inp["iif"] = 1
    inp["src_vni"] = VPC_C
    return buf, inp, int(pf.sum())
