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


def masq_tables(genid: int = 1, pool: str = "203.0.113.0/24") -> TB:
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
    t.add_masquerade(VPC_C, VPC_S, ["10.0.0.0/8"], [pool])
    t.add_ff_remote(VPC_C, "198.18.0.0/15", VPC_S)
    t.add_ff_remote(VPC_C, "198.18.0.0/15", VPC_S, gate_vni=VPC_S)
    t.add_ff_local(VPC_C, VPC_S, "10.0.0.0/8", NAT_MASQUERADE)
    t.add_ff_remote(VPC_C, "172.16.0.0/12", VPC_P)
    t.add_ff_local(VPC_C, VPC_P, "10.0.0.0/8")
    return t


def masq_world(genid: int = 1, pool: str = "203.0.113.0/24") -> TB:
    """masq_tables with the way back: VPC 200's answers to the public pool
    (203.0.113.0/24, gated on VPC 100, requiring masquerade) reach VPC 100's
    clients -- the reference's lowering of a masquerading peering's return
    direction (flow-filter/src/context/tables.rs:583-662).  `pool`: a part of
    203.0.113.0/24 as the public pool instead (a small pool runs out)."""
    t = masq_tables(genid, pool)
    t.add_ff_remote(VPC_S, pool, VPC_C, NAT_MASQUERADE, gate_vni=VPC_C)
    t.add_ff_local(VPC_S, VPC_C, "198.18.0.0/15")
    return t


def _ip(a: np.ndarray) -> np.ndarray:
    """u32 addresses -> (n, 4) big-endian bytes"""
    return a.astype(">u4").view(np.uint8).reshape(-1, 4)


def frames(src, dst, sport, dport, vni):
    """(buf, inp): 64-byte Ethernet / IPv4 / UDP frames in SLOT-byte slots,
    one per row of the u32 / u16 arrays, arriving in VPC `vni` (per packet)."""
    n = len(src)
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
    ip[:, 12:16] = _ip(np.asarray(src, np.uint32))
    ip[:, 16:20] = _ip(np.asarray(dst, np.uint32))
    words = ip.reshape(n, 10, 2).astype(np.uint32)
    s = (words[:, :, 0] << 8 | words[:, :, 1]).sum(axis=1)
    s = (s & 0xffff) + (s >> 16)
    s = (s & 0xffff) + (s >> 16)
    ck = (~s & 0xffff).astype(np.uint16)
    ip[:, 10] = ck >> 8
    ip[:, 11] = ck & 0xff
    udp = fr[:, 34:42]
    udp[:, 0:2] = np.asarray(sport, np.uint16).astype(">u2").view(np.uint8).reshape(-1, 2)
    udp[:, 2:4] = np.asarray(dport, np.uint16).astype(">u2").view(np.uint8).reshape(-1, 2)
    udp[:, 4:6] = np.array([0, FRAME - 34], np.uint8)  # checksum 0: none (IPv4)
    head = SLOT - FRAME
    buf = np.zeros(n * SLOT + 64, dtype=np.uint8)
    buf[: n * SLOT].reshape(n, SLOT)[:, head:] = fr
    inp = np.zeros(n, dtype=A.PKT_IN)
    inp["off"] = np.arange(n, dtype=np.uint32) * SLOT + head
    inp["len"] = FRAME
    inp["flags"] = A.IN_SEEDED_OVERLAY
    inp["iif"] = 1
    inp["src_vni"] = vni
    return buf, inp


class MasqConns:
    """`e` masqueraded UDP connections of masq_world (VPC 100 clients in
    10.250.0.0/16 to VPC 200 servers in 198.18.0.0/15) for the masquerade-heavy
    bursts: their first packets (every one allocates a tuple), then bursts in
    which nearly every packet belongs to one of them -- the client's packets
    and the server's answers to the public tuple -- beside a share of new
    connections."""

    def __init__(self, e: int, seed: int = 7):
        rng = np.random.default_rng(seed)
        idx = np.arange(e, dtype=np.uint64)
        self.e = e
        self.src = (np.uint64(10 << 24 | 250 << 16) + (idx >> np.uint64(6))).astype(np.uint32)
        self.sport = (1024 + (idx & np.uint64(63)) * 900 + np.uint64(7)).astype(np.uint16)
        self.dst = (np.uint32(198 << 24 | 18 << 16) + rng.integers(1, 1 << 17, e).astype(np.uint32))
        dp = rng.integers(1000, 65535, e)
        self.dport = np.where(np.isin(dp, (53, 853, 8853)), dp + 1, dp).astype(np.uint16)
        self.pub = np.zeros(e, np.uint32)    # the public tuple each was given (learn)
        self.pport = np.zeros(e, np.uint16)

    def first(self):
        """(buf, inp): every connection's first packet, in order."""
        return frames(self.src, self.dst, self.sport, self.dport, VPC_C)

    def learn(self, buf: np.ndarray, out: np.ndarray) -> int:
        """The public tuples from the delivered first packets; returns how many."""
        ok = out["done"] == A.DONE["Delivered"]
        k = np.nonzero(ok)[0]
        off = out["off"][k].astype(np.int64)
        b = lambda o: buf[off + o].astype(np.uint32)
        self.pub[k] = (b(26) << 24) | (b(27) << 16) | (b(28) << 8) | b(29)
        self.pport[k] = ((b(34) << 8) | b(35)).astype(np.uint16)
        return len(k)

    def keys(self):
        """Each connection's forward flow key (FlowKey, dp_flow_key_t)."""
        k = np.zeros(self.e, A.FLOW_KEY)
        k["src_vni"], k["family"], k["kind"] = VPC_C, 4, A.FLOW_UDP
        k["sport"], k["dport"] = self.sport, self.dport
        k["src"][:, :4] = _ip(self.src)
        k["dst"][:, :4] = _ip(self.dst)
        return k

    def burst(self, n: int, new_share: float, fwd_share: float, step: int, seed: int = 1):
        """(buf, inp, n_new): n packets in random order -- a share of them first
        packets of new connections (distinct clients 10.<step>.x.y), the rest
        on the learnt connections, the client's (fwd_share) or the server's."""
        rng = np.random.default_rng(seed * 7919 + step)
        nn = int(round(n * new_share))
        ne = n - nn
        c = rng.integers(0, self.e, ne)
        fwd = (rng.random(ne) < fwd_share) | (self.pport[c] == 0)  # answers only where a tuple was learnt
        src = np.where(fwd, self.src[c], self.dst[c])
        dst = np.where(fwd, self.dst[c], self.pub[c])
        sp = np.where(fwd, self.sport[c], self.dport[c])
        dpt = np.where(fwd, self.dport[c], self.pport[c])
        vni = np.where(fwd, VPC_C, VPC_S)
        j = np.arange(nn, dtype=np.uint64)
        nsrc = (np.uint64(10 << 24) + np.uint64((step % 200) << 16) + (j >> np.uint64(6))).astype(np.uint32)
        nsp = (1024 + (j & np.uint64(63)) * 900 + np.uint64(step % 900)).astype(np.uint16)
        ndst = (np.uint32(198 << 24 | 18 << 16) + rng.integers(1, 1 << 17, nn).astype(np.uint32))
        ndp = rng.integers(1000, 50000, nn).astype(np.uint16)
        allsrc = np.concatenate([src, nsrc]).astype(np.uint32)
        alldst = np.concatenate([dst, ndst]).astype(np.uint32)
        allsp = np.concatenate([sp, nsp]).astype(np.uint16)
        alldp = np.concatenate([dpt, ndp]).astype(np.uint16)
        allvni = np.concatenate([vni, np.full(nn, VPC_C)]).astype(np.uint32)
        perm = rng.permutation(len(allsrc))
        buf, inp = frames(allsrc[perm], alldst[perm], allsp[perm], alldp[perm], allvni[perm])
        return buf, inp, nn


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


# ---------------------------------------------------------------------------
# Port forwarding and masquerade on one public range (the reference's
# overlapping-expose configuration, nat/src/test.rs:141-174, scaled up)
# ---------------------------------------------------------------------------
MIX_PUB = "203.0.113.0/24"
MIX_PF_PORTS, MIX_INT_PORTS = (3000, 3999), (5000, 5999)


def mixed_world(genid: int = 1) -> TB:
    """VPC 200 (internal) masquerades 198.18.0.0/15 behind 203.0.113.0/24
    towards VPC 100 (external, clients 10.0.0.0/8) and forwards
    203.0.113.0/24 ports 3000-3999 (TCP and UDP) onto 198.18.0.0/24 ports
    5000-5999 -- the masquerade pool's own addresses, the forwarded ports
    claimed from it (apalloc/setup.rs:73-91).  Lowered as the reference lowers
    the overlay (flow-filter/src/context/tables.rs:566-676; tests/golden/
    natcombo.py does the same for nat/src/test.rs): VPC 100 reaches the public
    range as port forwarding (ungated, the priority tie bit) and as masquerade
    (gated on VPC 200: replies only); VPC 200's sources masquerade, its
    forwarded hosts answer only on their flows (gated on PortFwdReply).  VPC
    100 also routes 172.16.0.0/12 to VPC 300 without NAT."""
    t = TB(genid=genid)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    for v in (VPC_C, VPC_S, VPC_P):
        t.add_route(t.add_fib(v, vnis=[v]), "0.0.0.0/0", nh)
    t.add_ff_remote(VPC_C, MIX_PUB, VPC_S, NAT_MASQUERADE, gate_vni=VPC_S)
    t.add_ff_remote(VPC_C, MIX_PUB, VPC_S, NAT_PORT_FORWARDING, dports=MIX_PF_PORTS, port_forwarding=True)
    t.add_ff_local(VPC_C, VPC_S, "10.0.0.0/8")
    t.add_ff_remote(VPC_C, "172.16.0.0/12", VPC_P)
    t.add_ff_local(VPC_C, VPC_P, "10.0.0.0/8")
    t.add_ff_remote(VPC_S, "10.0.0.0/8", VPC_C)
    t.add_ff_local(VPC_S, VPC_C, "198.18.0.0/15", NAT_MASQUERADE)
    t.add_ff_local(VPC_S, VPC_C, "198.18.0.0/24", NAT_PORT_FORWARDING, sports=MIX_INT_PORTS, gate=1)
    for proto in (6, 17):
        t.add_portfw(src_vni=VPC_C, proto=proto, dst_vni=VPC_S, ext_prefix=MIX_PUB, int_prefix="198.18.0.0/24",
                     ext_ports=MIX_PF_PORTS, int_ports=MIX_INT_PORTS)
    t.add_masquerade(VPC_S, VPC_C, ["198.18.0.0/15"], [MIX_PUB],
                     claims=[(MIX_PUB, MIX_PF_PORTS[0], MIX_PF_PORTS[1], A.MASQ_TCP | A.MASQ_UDP)])
    return t


def _u32(a) -> np.ndarray:
    return np.asarray(a, dtype=np.uint64).astype(np.uint32)


class MixedConns:
    """Connections of mixed_world: `e_pf` port-forwarded ones (client
    10.1.x.y:p to 203.0.113.k:3000-3999, forwarded to 198.18.0.k:5000-5999)
    and `e_m` masqueraded ones (internal 198.18.128.0/17 hosts to external
    10.2.0.0/16 servers).  first(): every connection's first packet; then
    bursts in which a share opens new connections of both kinds and the rest
    belongs to the known ones -- each side's packets and the answers (the
    forwarded hosts' replies, the servers' answers to the public tuples)."""

    def __init__(self, e_pf: int, e_m: int, seed: int = 11):
        rng = np.random.default_rng(seed)
        self.e_pf, self.e_m = e_pf, e_m
        i = np.arange(e_pf, dtype=np.uint64)
        self.pf_src = _u32((10 << 24 | 1 << 16) + (i >> np.uint64(4)))
        self.pf_sport = (2000 + (i & np.uint64(15)) * 3000 + np.uint64(11)).astype(np.uint16)
        k = rng.integers(0, 256, e_pf).astype(np.uint32)
        self.pf_dst = _u32((203 << 24 | 0 << 16 | 113 << 8)) + k
        self.pf_dport = rng.integers(MIX_PF_PORTS[0], MIX_PF_PORTS[1] + 1, e_pf).astype(np.uint16)
        # where the rule forwards them (PortFwEntry::map_address_port)
        self.pf_int = _u32(198 << 24 | 18 << 16) + k
        self.pf_iport = (self.pf_dport.astype(np.uint32) - MIX_PF_PORTS[0] + MIX_INT_PORTS[0]).astype(np.uint16)
        j = np.arange(e_m, dtype=np.uint64)
        self.m_src = _u32((198 << 24 | 18 << 16 | 128 << 8) + (j >> np.uint64(5)))
        self.m_sport = (1024 + (j & np.uint64(31)) * 1900 + np.uint64(3)).astype(np.uint16)
        self.m_dst = _u32(10 << 24 | 2 << 16) + rng.integers(1, 1 << 16, e_m).astype(np.uint32)
        dp = rng.integers(1000, 65535, e_m)
        self.m_dport = np.where(np.isin(dp, (53, 853, 8853)), dp + 1, dp).astype(np.uint16)
        self.pub = np.zeros(e_m, np.uint32)
        self.pport = np.zeros(e_m, np.uint16)

    def first(self):
        """(buf, inp): the port-forwarded connections' first packets, then the
        masqueraded ones'."""
        src = np.concatenate([self.pf_src, self.m_src])
        dst = np.concatenate([self.pf_dst, self.m_dst])
        sp = np.concatenate([self.pf_sport, self.m_sport])
        dp = np.concatenate([self.pf_dport, self.m_dport])
        vni = np.concatenate([np.full(self.e_pf, VPC_C), np.full(self.e_m, VPC_S)]).astype(np.uint32)
        return frames(src, dst, sp, dp, vni)

    def learn(self, buf: np.ndarray, out: np.ndarray) -> int:
        """The public tuples of the delivered masqueraded first packets (first()'s order)."""
        o = out[self.e_pf:]
        k = np.nonzero(o["done"] == A.DONE["Delivered"])[0]
        off = o["off"][k].astype(np.int64)
        b = lambda x: buf[off + x].astype(np.uint32)
        self.pub[k] = (b(26) << 24) | (b(27) << 16) | (b(28) << 8) | b(29)
        self.pport[k] = ((b(34) << 8) | b(35)).astype(np.uint16)
        return len(k)

    def keys(self):
        """Every connection's forward flow key (port-forwarded, then masqueraded)."""
        k = np.zeros(self.e_pf + self.e_m, A.FLOW_KEY)
        k["family"], k["kind"] = 4, A.FLOW_UDP
        k["src_vni"][: self.e_pf], k["src_vni"][self.e_pf:] = VPC_C, VPC_S
        k["sport"] = np.concatenate([self.pf_sport, self.m_sport])
        k["dport"] = np.concatenate([self.pf_dport, self.m_dport])
        k["src"][:, :4] = _ip(np.concatenate([self.pf_src, self.m_src]))
        k["dst"][:, :4] = _ip(np.concatenate([self.pf_dst, self.m_dst]))
        return k

    def burst(self, n: int, new_share: float, step: int, seed: int = 1, answer_share: float = 0.4,
              pf_share: float = 0.5, same_burst_replies: int = 0):
        """(buf, inp, n_new_pf, n_new_m): n packets in random order -- new_share
        of them first packets of new connections (half port-forwarded from
        fresh clients 10.<100+step>.x.y, half masqueraded from fresh internal
        ports), the rest on the known connections (pf_share of them
        port-forwarded), answer_share of those the answers.
        same_burst_replies: that many forwarded hosts answer a new
        connection in the very burst that opens it (their packets masquerade
        on a key the creation inserts: the burst runs on one lane)."""
        rng = np.random.default_rng(seed * 7919 + step)
        nn = int(round(n * new_share))
        npf_new, nm_new = nn // 2, nn - nn // 2
        ne = n - nn - same_burst_replies
        is_pf = rng.random(ne) < pf_share
        ans = rng.random(ne) < answer_share
        cp = rng.integers(0, self.e_pf, ne)
        cm = rng.integers(0, self.e_m, ne)
        ans_m = ans & (self.pport[cm] != 0)  # (answers only where a tuple was learnt)
        src = np.where(is_pf, np.where(ans, self.pf_int[cp], self.pf_src[cp]),
                       np.where(ans_m, self.m_dst[cm], self.m_src[cm]))
        dst = np.where(is_pf, np.where(ans, self.pf_src[cp], self.pf_dst[cp]),
                       np.where(ans_m, self.pub[cm], self.m_dst[cm]))
        sp = np.where(is_pf, np.where(ans, self.pf_iport[cp], self.pf_sport[cp]),
                      np.where(ans_m, self.m_dport[cm], self.m_sport[cm]))
        dp = np.where(is_pf, np.where(ans, self.pf_sport[cp], self.pf_dport[cp]),
                      np.where(ans_m, self.pport[cm], self.m_dport[cm]))
        vni = np.where(is_pf, np.where(ans, VPC_S, VPC_C), np.where(ans_m, VPC_C, VPC_S))
        # new port-forwarded connections: fresh clients, one port each
        j = np.arange(npf_new, dtype=np.uint64)
        k = rng.integers(0, 256, npf_new).astype(np.uint32)
        nps = _u32((10 << 24) + ((100 + step % 100) << 16) + (j >> np.uint64(4)))
        npp = (2000 + (j & np.uint64(15)) * 3000 + np.uint64(step % 2000)).astype(np.uint16)
        npd = _u32(203 << 24 | 113 << 8) + k
        npdp = rng.integers(MIX_PF_PORTS[0], MIX_PF_PORTS[1] + 1, npf_new).astype(np.uint16)
        # new masqueraded connections: fresh internal sources (198.18.64.0/18)
        j = np.arange(nm_new, dtype=np.uint64)
        nms = _u32((198 << 24 | 18 << 16 | 64 << 8) + (j >> np.uint64(5)) + np.uint64((step % 8) << 11))
        nmp = (1024 + (j & np.uint64(31)) * 1900 + np.uint64(step % 1900)).astype(np.uint16)
        nmd = _u32(10 << 24 | 2 << 16) + rng.integers(1, 1 << 16, nm_new).astype(np.uint32)
        nmdp = rng.integers(1000, 50000, nm_new).astype(np.uint16)
        # the forwarded hosts answering new connections of this very burst
        r = min(same_burst_replies, npf_new)
        rs = _u32(198 << 24 | 18 << 16) + k[:r]
        rp = (npdp[:r].astype(np.uint32) - MIX_PF_PORTS[0] + MIX_INT_PORTS[0]).astype(np.uint16)
        allsrc = np.concatenate([src, nps, nms, rs]).astype(np.uint32)
        alldst = np.concatenate([dst, npd, nmd, nps[:r]]).astype(np.uint32)
        allsp = np.concatenate([sp, npp, nmp, rp]).astype(np.uint16)
        alldp = np.concatenate([dp, npdp, nmdp, npp[:r]]).astype(np.uint16)
        allvni = np.concatenate([vni, np.full(npf_new, VPC_C), np.full(nm_new, VPC_S),
                                 np.full(r, VPC_S)]).astype(np.uint32)
        perm = rng.permutation(len(allsrc))
        if r:
            # each reply after the packet that opens its connection
            pos = np.empty(len(perm), np.int64)
            pos[perm] = np.arange(len(perm))
            a = ne + np.arange(r)                      # the openers' rows
            b = ne + npf_new + nm_new + np.arange(r)   # the replies' rows
            lo, hi = np.minimum(pos[a], pos[b]), np.maximum(pos[a], pos[b])
            perm[lo], perm[hi] = a, b
        buf, inp = frames(allsrc[perm], alldst[perm], allsp[perm], alldp[perm], allvni[perm])
        return buf, inp, npf_new, nm_new
