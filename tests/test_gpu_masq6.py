"""GPU: masquerade over IPv6 (NAT66; the allocator's 128-bit regions,
nat/src/masquerade/apalloc/mod.rs, alloc.rs) against the oracle -- the
reference's masquerade tests are all IPv4, so these seeded bursts are the
v6 coverage: UDP and TCP connections from a private /64 masqueraded behind
a public /120 pool (two VPCs sharing it), then the peers' replies built
from the translated packets, repeats and closes; every burst bit-exact
(records, bytes) and the flow counts equal.  Parity against the oracle
only (no reference fixture holds a v6 masquerade case)."""
import ipaddress
import random
import struct

import numpy as np
import pytest

import pktgen as P
from dataplane_amd import _abi as A
from dataplane_amd.tables import NAT_MASQUERADE, TablesBuilder as TB
from edgecase import pack_burst
from golden.kat import IF_MAC, NH_MAC, OIF_MAC, PEER_MAC
from helpers import compare

pytestmark = pytest.mark.gpu

V1, V2, V3 = 1001, 1002, 1003


def world():
    t = TB(genid=1)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    for v in (V1, V2, V3):
        f = t.add_fib(v, vnis=[v])
        t.add_route(f, "0.0.0.0/0", nh)
        t.add_route(f, "::/0", nh)
    t.add_masquerade(V1, V2, ["fd00:1::/64"], ["2001:db8:100::/120"], idle_timeout_s=30)
    t.add_masquerade(V3, V2, ["fd00:3::/64"], ["2001:db8:100::/120"])
    for s in (V1, V3):
        t.add_ff_remote(s, "::/0", V2)
        t.add_ff_remote(s, "::/0", V2, gate_vni=V2)
        t.add_ff_local(s, V2, "::/0", NAT_MASQUERADE)
        t.add_ff_remote(V2, "::/0", s)
        t.add_ff_remote(V2, "::/0", s, gate_vni=s)
        t.add_ff_local(V2, s, "::/0")
    return t.build()


def frame(src, dst, proto, sport, dport, flags=0):
    if proto == 6:
        body = P.tcp(sport, dport, b"", P.pseudo6(src, dst, 6, 20), flags=flags)
    else:
        body = P.udp(sport, dport, b"", P.pseudo6(src, dst, 17, 8))
    return P.eth(IF_MAC, PEER_MAC, 0x86DD) + P.ipv6(src, dst, proto, len(body)) + body


def fields(fr: bytes):
    src = str(ipaddress.ip_address(fr[22:38]))
    dst = str(ipaddress.ip_address(fr[38:54]))
    sport, dport = struct.unpack("!HH", fr[54:58])
    return src, dst, sport, dport


@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_masquerade_v6_bursts(seed):
    import torch
    torch.cuda.init()
    from dataplane_amd import GpuPathNf
    from dataplane_amd.flows import FlowTable
    from oracle.pyoracle import Oracle, OracleFlows
    tp = world()
    rng = random.Random(seed)
    conns = []
    for k in range(600):
        vni = V1 if rng.random() < 0.6 else V3
        net = "fd00:1::" if vni == V1 else "fd00:3::"
        proto = 6 if rng.random() < 0.5 else 17
        conns.append((vni, f"{net}{k + 1:x}", f"2001:db8:200::{rng.randrange(1, 200):x}", proto,
                      1024 + rng.randrange(60000), 80 + rng.randrange(4)))
    o, oft = Oracle(tp), OracleFlows()
    nf, gft = GpuPathNf(0), FlowTable(0, 1 << 14)
    outs = {}
    SYN, ACK, FIN = 0x02, 0x10, 0x01
    try:
        nf.publish(tp)
        nf.attach_flows(gft)
        for step in range(3):
            pk, who = [], []
            for c, (vni, src, dst, proto, sp, dp) in enumerate(conns):
                if step == 0:
                    pk.append((frame(src, dst, proto, sp, dp, SYN if proto == 6 else 0), vni))
                    who.append((c, "fwd"))
                    if rng.random() < 0.1:  # the first packet twice: the second pair replaces the first
                        pk.append((frame(src, dst, proto, sp, dp, SYN if proto == 6 else 0), vni))
                        who.append((c, "fwd"))
                elif c in outs:
                    osrc, odst, osp, odp = outs[c]
                    pk.append((frame(odst, osrc, proto, odp, osp, (SYN | ACK) if proto == 6 else 0), V2))
                    who.append((c, "rev"))
                    fl = (FIN | ACK) if (proto == 6 and step == 2 and rng.random() < 0.3) else ACK
                    pk.append((frame(src, dst, proto, sp, dp, fl if proto == 6 else 0), vni))
                    who.append((c, "fwd"))
            order = list(range(len(pk)))
            rng.shuffle(order)
            pk = [pk[i] for i in order]
            who = [who[i] for i in order]
            buf, inp = pack_burst([(f, 1, A.IN_SEEDED_OVERLAY, v) for f, v in pk])
            ob, gb = buf.copy(), buf.copy()
            oout, _ = o.process_flows(ob, inp, oft)
            gout = nf.process_arrays(gb, inp)
            compare(oout, ob, gout, gb, inp, f"v6 masquerade seed {seed} burst {step}")
            assert gft.count() == oft.count(), f"burst {step}: counts"
            delivered = 0
            pool = ipaddress.ip_network("2001:db8:100::/120")
            for i, (c, d) in enumerate(who):
                r = oout[i]
                if r["done"] != A.DONE["Delivered"]:
                    continue
                delivered += 1
                if d == "fwd":
                    f = fields(ob[r["off"]:r["off"] + r["len"]].tobytes())
                    assert ipaddress.ip_address(f[0]) in pool, f"burst {step}: source {f[0]} not masqueraded"
                    outs[c] = f
            assert delivered > len(conns) // 2, f"burst {step}: {delivered} delivered"
    finally:
        nf.attach_flows(None)
        gft.close()
        nf.close()
