"""Edge-case corpus for the parity tests.

``edge_tables()`` lowers a small configuration that reaches every branch of the
path: interfaces in every admin/oper/type/attach state, an underlay FIB with
drop / local / ECMP / unresolved / zero-MAC / no-ifindex routes, VPC FIBs with
VXLAN encap (with and without dmac, v4 and v6 VTEPs), two-stage flow-filter
tables with port ranges and protocols, first-match ACLs with defaults, and
static NAT tables with NAT and PAT entries (including a multicast target, and
a PAT range that reaches port 0).

``edge_burst(n, seed)`` draws frames from templates aimed at those tables and
then mutates them: truncation, random byte flips in the header region,
malformed header fields (IHL, versions, ports, doff, VIDs, VXLAN flags, AH
lengths), extension chains over the MAX_NET_EXTENSIONS limit, VLAN stacks
over MAX_VLANS, TTL 0/1, broadcast / foreign / zero MACs, unknown interfaces,
seeded overlay packets from known and unknown VNIs.
"""
from __future__ import annotations

import random
import struct

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.tables import (ALLOW, ATTACH_BRIDGE, ATTACH_NONE, DENY, IF_DOWN, IF_UNKNOWN,
                                  IFT_LOOPBACK, IFT_VXLAN, IFT_DOT1Q, NAT_NONE, NAT_STATIC,
                                  TablesBuilder)
import pktgen as P

M1 = "02:00:00:00:00:01"          # iif 1 (underlay, VRF 0)
PEER = "02:00:00:00:ee:01"
VTEP4 = "100.64.0.1"
VTEP6 = "2001:db8:ffff::1"
TB = TablesBuilder


def edge_tables() -> TablesBuilder:
    t = TablesBuilder(genid=7)
    # ---- interfaces
    t.add_iface(1, M1)
    t.add_iface(2, "02:00:00:00:00:02", admin=IF_DOWN)
    t.add_iface(3, "02:00:00:00:00:03", oper=IF_DOWN)           # ingress ignores oper state
    t.add_iface(4, "02:00:00:00:00:04", attach=ATTACH_BRIDGE)
    t.add_iface(5, "02:00:00:00:00:05", attach=ATTACH_NONE)
    t.add_iface(6, "02:00:00:00:00:06", iftype=IFT_LOOPBACK)
    t.add_iface(7, "02:00:00:00:00:07", admin=IF_UNKNOWN, iftype=IFT_DOT1Q)
    t.add_iface(8, "02:00:00:00:00:08", vrf_id=9)              # VRF without a FIB
    t.add_iface(9, "02:00:00:00:00:09", vrf_id=100)            # directly in a VPC VRF
    t.add_iface(10, "02:00:00:00:00:10")
    t.add_iface(11, "02:00:00:00:00:11", admin=IF_DOWN)
    t.add_iface(12, "02:00:00:00:00:12", oper=IF_DOWN)
    t.add_iface(13, "02:00:00:00:00:13", iftype=IFT_VXLAN)
    t.add_iface(14, "02:00:00:00:00:14", iftype=IFT_DOT1Q)
    # ---- adjacencies
    t.add_adjacency("192.0.2.1", 10, "02:00:00:00:77:01")
    t.add_adjacency("192.0.2.2", 11, "02:00:00:00:77:02")
    t.add_adjacency("192.0.2.3", 12, "02:00:00:00:77:03")
    t.add_adjacency("192.0.2.4", 13, "02:00:00:00:77:04")
    t.add_adjacency("192.0.2.5", 14, "02:00:00:00:77:05")
    t.add_adjacency("192.0.2.6", 15, "02:00:00:00:77:06")   # oif 15 unknown
    t.add_adjacency("192.0.2.77", 10, "00:00:00:00:00:00")  # resolved to a zero MAC
    t.add_adjacency("192.0.2.1", 14, "02:00:00:00:77:41")   # same ip, other oif
    for k in range(1, 8):
        t.add_adjacency(f"198.51.100.{k}", 10, f"02:00:00:00:66:{k:02x}")
    t.add_adjacency("2001:db8::1", 10, "02:00:00:00:76:01")
    t.add_adjacency("2001:db8:2::5", 10, "02:00:00:00:76:05")
    # ---- FIBs
    und = t.add_fib(0, vtep_ip=VTEP4, vtep_mac=M1)
    vpc = {}
    vpc[1000] = t.add_fib(100, vtep_ip=VTEP4, vtep_mac=M1, vnis=[1000])
    vpc[1001] = t.add_fib(101, vtep_ip=VTEP4, vtep_mac=M1, vnis=[1001])
    vpc[1002] = t.add_fib(102, vnis=[1002])
    vpc[2000] = t.add_fib(200, vtep_ip=VTEP4, vtep_mac=M1, vnis=[2000])
    vpc[2001] = t.add_fib(201, vtep_ip=VTEP6, vtep_mac=M1, vnis=[2001])  # v6 VTEP
    vpc[2002] = t.add_fib(202, vtep_ip=VTEP4, vnis=[2002])               # no VTEP mac
    vpc[2003] = t.add_fib(203, vtep_ip=VTEP4, vtep_mac="03:00:00:00:00:01", vnis=[2003])
    vpc[2004] = t.add_fib(204, vtep_mac=M1, vnis=[2004])                 # no VTEP ip
    vpc[2005] = t.add_fib(205, vtep_ip="224.0.0.9", vtep_mac=M1, vnis=[2005])
    # ---- next hops
    eg = lambda oif, a=None: t.add_nh([[TB.egress(oif, a)]])  # noqa: E731
    nh_drop = t.add_nh([[TB.drop()]])
    nh_local = t.add_nh([[TB.local(1)]])
    nh_a = eg(10, "192.0.2.1")
    # underlay
    t.add_route(und, "0.0.0.0/0", nh_drop)
    t.add_route(und, "192.0.2.0/24", nh_a)
    t.add_route(und, "198.51.100.0/24", eg(10))                 # connected: adjacency by dst
    t.add_route(und, "203.0.113.0/26", eg(11, "192.0.2.2"))     # admin down
    t.add_route(und, "203.0.113.64/26", eg(12, "192.0.2.3"))    # oper down
    t.add_route(und, "203.0.113.128/26", eg(13, "192.0.2.4"))   # unsupported type
    t.add_route(und, "203.0.113.192/27", eg(14, "192.0.2.5"))   # dot1q ok
    t.add_route(und, "203.0.113.224/27", eg(15, "192.0.2.6"))   # unknown oif
    t.add_route(und, "198.18.0.0/15", t.add_nh([[TB.egress(10, "192.0.2.1")],
                                               [TB.egress(14, "192.0.2.5")],
                                               [TB.egress(14, "192.0.2.1")],
                                               [TB.drop()]]))      # ECMP x4
    t.add_route(und, "198.19.0.0/16", eg(None, "192.0.2.1"))    # no ifindex
    t.add_route(und, "198.19.1.0/24", eg(10, "192.0.2.99"))     # unresolved
    t.add_route(und, "198.19.2.0/24", eg(10, "192.0.2.77"))     # zero MAC
    t.add_route(und, "198.19.3.0/24", t.add_nh([[TB.egress(10, "192.0.2.1"),
                                                TB.egress(14, "192.0.2.5")]]))  # last wins
    t.add_route(und, "198.19.4.128/25", t.add_nh([[TB.egress(10), TB.drop()]]))
    t.add_route(und, VTEP4 + "/32", nh_local)
    t.add_route(und, "100.64.0.0/10", nh_a)
    t.add_route(und, "100.65.0.0/16", eg(10, "192.0.2.1"))
    t.add_route(und, "10.255.0.0/16", nh_drop)
    t.add_route(und, "10.0.0.0/8", nh_a)
    t.add_route(und, "::/0", nh_drop)
    t.add_route(und, "2001:db8:1::/48", eg(10, "2001:db8::1"))
    t.add_route(und, "2001:db8:2::/48", eg(10))
    t.add_route(und, "2001:db8:3::/64", t.add_nh([[TB.egress(10, "2001:db8::1")],
                                                 [TB.egress(10, "192.0.2.1")]]))
    t.add_route(und, "2001:db8:4::/48", t.add_nh([[TB.local(1)]]))
    t.add_route(und, "2001:db8:4:1::/64", eg(10, "192.0.2.1"))
    # the VPC reached directly from iif 9 (VRF 100)
    t.add_route(vpc[1000], "0.0.0.0/0", nh_drop)
    t.add_route(vpc[1000], "10.0.0.0/8", nh_a)
    t.add_route(vpc[1000], "::/0", nh_drop)
    t.add_route(vpc[1001], "0.0.0.0/0", nh_drop)
    # destination VPCs
    enc = lambda vni, rem, dmac="02:00:00:00:88:01", oif=10, a="192.0.2.1": t.add_nh(  # noqa: E731
        [[TB.encap(vni, rem, dmac), TB.egress(oif, a)]])
    d = vpc[2000]
    t.add_route(d, "0.0.0.0/0", enc(2000, "100.65.0.2"))
    t.add_route(d, "10.128.0.0/16", enc(2000, "100.65.0.3"))
    t.add_route(d, "10.129.0.0/16", enc(2000, "100.65.0.4", dmac=None))
    t.add_route(d, "10.129.1.0/24", enc(2000, "100.65.0.4", dmac="00:00:00:00:00:00"))
    t.add_route(d, "10.130.0.0/16", eg(10, "192.0.2.1"))          # plain egress, no encap
    t.add_route(d, "10.131.0.0/16", nh_drop)
    t.add_route(d, "10.132.0.0/16", t.add_nh([[TB.encap(2000, "100.65.0.5", "02:00:00:00:88:05"),
                                              TB.egress(10, "192.0.2.1")],
                                             [TB.encap(2000, "100.65.0.6", "02:00:00:00:88:06"),
                                              TB.egress(14, "192.0.2.5")]]))
    t.add_route(d, "10.133.0.0/16", enc(2000, "2001:db8:9::1"))   # v4 VTEP, v6 remote
    t.add_route(d, "10.134.0.0/16", enc(2000, "100.65.0.7", oif=11, a="192.0.2.2"))
    t.add_route(d, "10.135.0.0/16", t.add_nh([[TB.encap(2000, "100.65.0.8", "02:00:00:00:88:08")]]))
    t.add_route(d, "10.136.0.0/16", enc(2000, "100.65.0.9", oif=10, a="192.0.2.99"))
    t.add_route(d, "::/0", enc(2000, "100.65.0.2"))
    t.add_route(d, "10.140.0.0/16", enc(2000, "100.65.0.10"))  # VPC 1010's NATed dsts
    t.add_route(d, "2001:db8:100::/48", eg(10, "2001:db8::1"))
    for vni in (2001, 2002, 2003, 2004, 2005):
        t.add_route(vpc[vni], "0.0.0.0/0", enc(vni, "100.65.0.2" if vni != 2001 else "2001:db8:9::2"))
        t.add_route(vpc[vni], "::/0", enc(vni, "100.65.0.2"))
    t.add_route(vpc[1002], "0.0.0.0/0", nh_drop)
    # ---- flow filter (remote: by dst; local: by src)
    for src in (1000, 1001):
        t.add_ff_remote(src, "172.32.0.0/16", 2000, NAT_STATIC)
        t.add_ff_remote(src, "10.128.0.0/12", 2000)
        t.add_ff_remote(src, "10.144.0.0/16", 2001, proto=6, dports=(80, 90))
        t.add_ff_remote(src, "10.144.0.0/16", 2002, proto=17)
        t.add_ff_remote(src, "10.145.0.0/16", 2003)
        t.add_ff_remote(src, "10.146.0.0/16", 2004)
        t.add_ff_remote(src, "10.147.0.0/16", 2005)
        t.add_ff_remote(src, "10.148.0.0/16", 1002)
        t.add_ff_remote(src, "2001:db8:100::/40", 2000)
    t.add_ff_remote(1000, "0.0.0.0/0", 2000)
    t.add_ff_remote(1000, "::/0", 2001)
    t.add_ff_remote(1000, "172.33.0.0/16", 2000, NAT_STATIC, proto=6, dports=(1, 1023))
    for dst in (2000, 2001, 2002, 2003, 2004, 2005, 1002):
        t.add_ff_local(1000, dst, "10.0.0.0/16", NAT_STATIC)
        t.add_ff_local(1000, dst, "10.1.0.0/16", NAT_STATIC, proto=6, sports=(1000, 2000))
        t.add_ff_local(1000, dst, "10.1.0.0/16", NAT_NONE, proto=17)
        t.add_ff_local(1000, dst, "0.0.0.0/0", NAT_NONE)
        t.add_ff_local(1000, dst, "::/0", NAT_NONE)
    t.add_ff_local(1001, 2000, "10.5.0.0/16", NAT_STATIC)
    # ---- ACL: first match in insertion order; defaults per VPC pair
    t.add_acl(1000, 2000, DENY, proto=17, dports=(53, 53))
    t.add_acl(1000, 2000, ALLOW, proto=6, src="10.0.1.0/24")
    t.add_acl(1000, 2000, DENY, dst="10.128.5.0/24")
    t.add_acl(1000, 2000, ALLOW, proto=1)
    t.add_acl(1000, 2000, DENY, src="10.0.0.0/16", dports=(1000, 1999))
    t.add_acl(1000, 2000, DENY, src="10.0.3.0/24", sports=(7, 9), dst="10.128.0.0/10")
    t.add_acl(1000, 2001, ALLOW, proto=6)
    t.add_acl(1001, 2000, DENY, dst="10.128.7.0/24")
    t.add_acl(1000, 2000, DENY, family=6, dst="2001:db8:100:5::/64")
    t.add_acl(1000, 2001, DENY, family=6, proto=17, dports=(53, 53))
    t.add_acl_default(1000, 2000, ALLOW)
    t.add_acl_default(1000, 2001, DENY)
    t.add_acl_default(1001, 2003, DENY)
    # ---- static NAT (NAT44)
    def rng(olo, ohi, tlo, thi, off=0, olop=0, ohip=65535, tlop=0, thip=65535):
        return (olo, olop, ohi, ohip, tlo, thi, tlop, thip, off)
    t.add_nat_table(1, 1000, 2000, [
        dict(prefix="10.0.0.0/24", size=256, ranges=[rng("10.0.0.0", "10.0.0.255",
                                                         "172.16.0.0", "172.16.0.255")]),
        dict(prefix="10.0.1.0/24", pat=True, port_ranges=[(1000, 1999)], size=256 * 1000,
             ranges=[rng("10.0.1.0", "10.0.1.255", "172.16.1.0", "172.16.1.255", 0, 1000, 1999,
                         3000, 3999)]),
        dict(prefix="10.0.2.0/24", size=256, ranges=[rng("10.0.2.0", "10.0.2.255",
                                                         "224.0.9.0", "224.0.9.255")]),
        dict(prefix="10.0.3.0/25", size=64, ranges=[rng("10.0.3.0", "10.0.3.63",
                                                        "172.16.3.0", "172.16.3.63")]),
        dict(prefix="10.0.0.0/16", size=65536, ranges=[
            rng("10.0.0.0", "10.0.127.255", "172.17.0.0", "172.17.127.255", 0),
            rng("10.0.128.0", "10.0.255.255", "172.18.0.0", "172.18.127.255", 32768)]),
        dict(prefix="10.1.0.0/16", pat=True, port_ranges=[(0, 99), (1000, 1999)], size=65536 * 100,
             ranges=[rng("10.1.0.0", "10.1.255.255", "172.19.0.0", "172.19.0.255", 0, 0, 99,
                         0, 99)]),
    ])
    t.add_nat_table(0, 1000, 0, [
        dict(prefix="172.32.0.0/24", size=256, ranges=[rng("172.32.0.0", "172.32.0.255",
                                                           "10.128.0.0", "10.128.0.255")]),
        dict(prefix="172.32.1.0/24", pat=True, port_ranges=[(80, 80)], size=256,
             ranges=[rng("172.32.1.0", "172.32.1.255", "10.128.1.10", "10.128.1.10", 0, 80, 80,
                         8000, 8255)]),
        dict(prefix="172.32.2.0/23", size=512, ranges=[rng("172.32.2.0", "172.32.3.255",
                                                           "10.128.2.0", "10.128.3.255")]),
        dict(prefix="172.32.2.0/24", size=256, ranges=[rng("172.32.2.0", "172.32.2.255",
                                                           "10.130.2.0", "10.130.2.255")]),
        dict(prefix="172.33.0.0/16", pat=True, port_ranges=[(1, 1023)], size=65536 * 1023,
             ranges=[rng("172.33.0.0", "172.33.255.255", "10.128.9.0", "10.128.9.255", 0, 1,
                         1023, 1, 65535)]),
    ])
    t.add_nat_table(0, 1001, 0, [])
    # ---- VPCs 1010 / 1011 take the kernel's fast overlay path (one peer
    # only, and enough rules / NAT prefixes for multibit indexes)
    vpc[1010] = t.add_fib(110, vtep_ip=VTEP4, vtep_mac=M1, vnis=[1010])
    vpc[1011] = t.add_fib(111, vnis=[1011])
    t.add_route(vpc[1010], "0.0.0.0/0", nh_drop)
    t.add_route(vpc[1011], "0.0.0.0/0", nh_drop)
    for v in (1010, 1011):
        for k in range(24):
            t.add_ff_remote(v, f"172.40.{k}.0/24", 2000, NAT_STATIC if k % 3 else NAT_NONE,
                            proto=6 if k % 5 == 0 else None,
                            dports=(80, 90) if k % 7 == 0 else (0, 65535))
        t.add_ff_remote(v, "10.128.0.0/12", 2000)
        t.add_ff_remote(v, "172.32.0.0/16", 2000, NAT_STATIC)
        t.add_ff_remote(v, "::/0", 2000)
        for k in range(20):
            t.add_ff_local(v, 2000, f"10.20.{k}.0/24", NAT_STATIC if k % 4 != 3 else NAT_NONE,
                           proto=17 if k % 6 == 0 else None,
                           sports=(1000, 2000) if k % 5 == 0 else (0, 65535))
    t.add_ff_remote(1010, "0.0.0.0/0", 2000)          # 1011: no default (misses filtered)
    t.add_ff_local(1010, 2000, "10.0.0.0/16", NAT_STATIC)
    t.add_ff_local(1010, 2000, "0.0.0.0/0", NAT_NONE)
    t.add_ff_local(1010, 2000, "::/0", NAT_NONE)
    for k in range(24):
        # every rule names a destination (a /16 parent for k == 0): the
        # per-interval candidate lists stay short, so the group takes the
        # candidate-list form with a multibit dst index
        kw = {"dst": "172.40.0.0/16" if k == 0 else
              f"172.40.{k}.0/24" if k % 2 else f"172.40.{k}.128/25"}
        if k % 3 == 0:
            kw["src"] = f"10.20.{k}.0/24"
        if k % 5 == 0:
            kw["proto"] = 6 if k % 10 == 0 else 17
        if k % 7 == 0:
            kw["dports"] = (53, 53)
        if k % 11 == 0:
            kw["sports"] = (1000, 1999)
        t.add_acl(1010, 2000, DENY if k % 3 == 1 else ALLOW, **kw)
    t.add_acl(1010, 2000, ALLOW, dst="172.40.0.0/19")  # after the specific rules
    t.add_acl_default(1010, 2000, DENY)               # 1011: no ACL at all
    src_ents, dst_ents = [], []
    for k in range(18):
        if k == 4:
            src_ents.append(dict(prefix=f"10.20.{k}.0/24", pat=True, port_ranges=[(1000, 1999)],
                                 size=256 * 1000, ranges=[rng(f"10.20.{k}.0", f"10.20.{k}.255",
                                                              "172.51.0.0", "172.51.3.255", 0,
                                                              1000, 1999, 2000, 2249)]))
        elif k == 5:
            src_ents.append(dict(prefix=f"10.20.{k}.0/24", size=256,
                                 ranges=[rng(f"10.20.{k}.0", f"10.20.{k}.255", "224.0.7.0",
                                             "224.0.7.255")]))
        elif k == 6:
            src_ents.append(dict(prefix=f"10.20.{k}.0/24", size=256, ranges=[
                rng(f"10.20.{k}.0", f"10.20.{k}.99", "172.52.0.0", "172.52.0.99", 0),
                rng(f"10.20.{k}.100", f"10.20.{k}.255", "172.53.0.0", "172.53.0.155", 100)]))
        else:
            src_ents.append(dict(prefix=f"10.20.{k}.0/24", size=256,
                                 ranges=[rng(f"10.20.{k}.0", f"10.20.{k}.255", f"172.50.{k}.0",
                                             f"172.50.{k}.255")]))
    src_ents.append(dict(prefix="10.20.0.0/16", size=65536, ranges=[
        rng("10.20.0.0", "10.20.255.255", "172.54.0.0", "172.54.255.255")]))
    for k in range(18):
        if k == 2:
            dst_ents.append(dict(prefix=f"172.40.{k}.0/24", pat=True, port_ranges=[(80, 90)], size=256 * 11,
                                 ranges=[rng(f"172.40.{k}.0", f"172.40.{k}.255", "10.140.2.1",
                                             "10.140.2.1", 0, 80, 90, 9000, 11815)]))
        else:
            dst_ents.append(dict(prefix=f"172.40.{k}.0/24", size=256,
                                 ranges=[rng(f"172.40.{k}.0", f"172.40.{k}.255", f"10.140.{k}.0",
                                             f"10.140.{k}.255")]))
    t.add_nat_table(1, 1010, 2000, src_ents)
    t.add_nat_table(0, 1010, 0, dst_ents)
    return t


# --------------------------------------------------------------------------
# burst generator

def _pick(r: random.Random, xs):
    return xs[r.randrange(len(xs))]


UNDERLAY_V4 = ["192.0.2.9", "198.51.100.3", "198.51.100.9", "203.0.113.5", "203.0.113.70",
               "203.0.113.130", "203.0.113.200", "203.0.113.230", "198.18.7.1", "198.19.200.1",
               "198.19.1.5", "198.19.2.5", "198.19.3.1", "198.19.4.200", VTEP4, "100.64.9.9",
               "100.65.3.3", "10.255.1.1", "10.3.2.1", "8.8.8.8"]
UNDERLAY_V6 = ["2001:db8:1::9", "2001:db8:2::5", "2001:db8:2::6", "2001:db8:3::1",
               "2001:db8:4::1", "2001:db8:4:1::1", "2001:db8:77::1"]
OVERLAY_V4_DST = ["172.32.0.9", "172.32.1.7", "172.32.2.5", "172.32.3.5", "172.32.9.9",
                  "172.33.4.4", "10.128.5.3", "10.128.7.1", "10.128.0.1", "10.129.0.5",
                  "10.129.1.5", "10.130.0.7", "10.131.0.1", "10.132.0.2", "10.133.0.1",
                  "10.134.0.1", "10.135.0.1", "10.136.0.1", "10.144.0.1", "10.145.0.1",
                  "10.146.0.1", "10.147.0.1", "10.148.0.1", "10.200.0.1", "192.168.1.1",
                  "172.40.0.9", "172.40.2.5", "172.40.3.9", "172.40.5.1", "172.40.7.1",
                  "172.40.14.2", "172.40.21.7", "172.40.30.1", "10.140.9.9", "172.40.2.130",
                  "172.40.40.1"]
OVERLAY_V4_SRC = ["10.0.0.5", "10.0.1.200", "10.0.2.3", "10.0.3.9", "10.0.3.100", "10.0.77.7",
                  "10.0.200.1", "10.1.2.3", "10.5.0.1", "10.9.9.9", "10.20.1.5", "10.20.4.9",
                  "10.20.5.5", "10.20.6.120", "10.20.6.7", "10.20.12.2", "10.20.18.2", "10.20.30.1",
                  "10.20.4.77", "10.20.5.200", "10.20.4.1"]
OVERLAY_V6_DST = ["2001:db8:100:5::1", "2001:db8:100:6::1", "2001:db8:1ff::1", "2001:db8:9999::1"]
OVERLAY_V6_SRC = ["2001:db8:aa::1", "2001:db8:bb::2"]
FAST_V4_SRC = ["10.20.1.5", "10.20.2.9", "10.20.3.3", "10.20.4.9", "10.20.4.77", "10.20.5.5",
               "10.20.5.200", "10.20.6.7", "10.20.6.120", "10.20.12.2", "10.20.17.1",
               "10.20.18.2", "10.20.30.1", "10.0.7.7", "10.9.9.9"]
FAST_V4_DST = ["172.40.0.9", "172.40.1.1", "172.40.2.5", "172.40.2.130", "172.40.3.9",
               "172.40.4.4", "172.40.5.1", "172.40.7.1", "172.40.14.2", "172.40.17.3",
               "172.40.21.7", "172.40.30.1", "172.40.40.1", "10.140.9.9", "172.32.3.3",
               "10.129.0.5", "192.168.1.1"]
FAST_PORTS = [53, 79, 80, 85, 90, 91, 443, 999, 1000, 1500, 1999, 2000, 2001, 8080]
PORTS = [1, 7, 8, 53, 80, 85, 99, 100, 443, 999, 1000, 1500, 1999, 2000, 2001, 4789, 8080,
         65535]


def _ports(r):
    return _pick(r, PORTS) if r.random() < 0.7 else r.randrange(1, 65536)


# --- ICMP error messages carrying an embedded packet fragment --------------
# (net/src/headers/embedded.rs; nat/src/icmp_handler).  The fragment is the
# packet the error answers: usually the reverse of the outer addresses (so the
# overlay NAT translates it back), with a full or truncated transport header.

def _emb_transport(r, v6, isrc, idst):
    """(next header, transport bytes) of an embedded packet, maybe truncated."""
    kind = _pick(r, ["udp", "udp", "tcp", "tcp", "echo", "icmp", "other"])
    pay = bytes(r.randrange(256) for _ in range(_pick(r, [0, 0, 4, 12, 30])))
    ps = (P.pseudo6 if v6 else P.pseudo4)
    sp, dp = _pick(r, [53, 80, 443, 1234, 2000, 8080]), _pick(r, [53, 80, 443, 999, 2001, 5678])
    if kind == "udp":
        nh, t = 17, P.udp(sp, dp, pay, ps(isrc, idst, 17, 8 + len(pay)))
    elif kind == "tcp":
        opts = b"" if r.random() < 0.8 else bytes([1] * 4)
        nh, t = 6, P.tcp(sp, dp, pay, ps(isrc, idst, 6, 20 + len(opts) + len(pay)), options=opts,
                         reserved=r.choice([0, 0, 0, 0xE]))
    elif kind == "echo":
        typ = _pick(r, [128, 129]) if v6 else _pick(r, [8, 0, 13])
        rest = struct.pack("!HH", r.randrange(65536), r.randrange(65536))
        if typ == 13:
            rest += bytes(12)
        code = 0 if r.random() < 0.85 else 1
        nh = 58 if v6 else 1
        t = (P.icmp6(typ, code, rest, pay, isrc, idst) if v6 else P.icmp4(typ, code, rest, pay))
    elif kind == "icmp":
        nh = 58 if v6 else 1
        t = (P.icmp6(1, 4, bytes(4), pay, isrc, idst) if v6 else P.icmp4(3, 3, bytes(4), pay))
    else:
        nh, t = 47, bytes(r.randrange(256) for _ in range(12))
    cut = _pick(r, [None, None, None, None, 8, 6, 4, 3, 1])
    return nh, (t if cut is None else t[:cut])


def _emb_packet(r, v6, isrc, idst):
    """An embedded IP packet fragment: (bytes, byte ranges of its extension headers)."""
    nh, body = _emb_transport(r, v6, isrc, idst)
    exts = []
    if v6:
        for _ in range(_pick(r, [0, 0, 0, 1, 2, 3, 4])):
            kind = _pick(r, [0, 43, 60, 44, 51])
            if kind == 44:
                e = P.ext_frag(nh, ident=r.randrange(1 << 32), reserved=r.randrange(2) * 0x11)
            elif kind == 51:
                e = P.ext_auth(nh, payload_len=1, reserved=r.randrange(2) * 0x1234)
            else:
                e = P.ext_raw(nh, hdr_len=_pick(r, [0, 1]), fill=r.randrange(256))
            exts.insert(0, e)
            nh = kind
        ip = P.ipv6(isrc, idst, nh, sum(map(len, exts)) + len(body) + 40, hop=_pick(r, [1, 63]))
    else:
        if r.random() < 0.1:  # IPv4 AH in front of the transport
            exts.insert(0, P.ext_auth(nh, payload_len=1))
            nh = 51
        evil = r.random() < 0.1
        ip = P.ipv4(isrc, idst, nh, sum(map(len, exts)) + len(body) + r.randrange(0, 100),
                    ttl=_pick(r, [1, 63]), evil=evil, ident=r.randrange(65536),
                    options=b"" if r.random() < 0.9 else bytes([1] * 4))
        if r.random() < 0.08:  # a bad embedded IPv4 checksum
            ip = ip[:10] + bytes([ip[10] ^ 0x5a]) + ip[11:]
        if r.random() < 0.05:  # not an IPv4 header at all
            ip = bytes([0x7e]) + ip[1:]
    ext_ranges, o = [], len(ip)
    for e in exts:
        ext_ranges.append((o, o + len(e)))
        o += len(e)
    return ip + b"".join(exts) + body, ext_ranges


def _icmp_err(r, v6, src, dst):
    """An ICMP error message (the L4 body of the outer packet src -> dst)."""
    if r.random() < 0.7:  # answers a packet dst -> src, as a reply would
        isrc, idst = dst, src
    else:
        isrc = _pick(r, OVERLAY_V6_DST if v6 else OVERLAY_V4_DST)
        idst = _pick(r, OVERLAY_V6_SRC if v6 else OVERLAY_V4_SRC)
    emb, ext_ranges = _emb_packet(r, v6, isrc, idst)
    if v6:
        typ = _pick(r, [1, 1, 2, 3, 4])
        code = {1: _pick(r, [0, 3, 4, 6, 7]), 2: 0, 3: _pick(r, [0, 1, 2]),
                4: _pick(r, [0, 1, 10, 11])}[typ]
        rest = (struct.pack("!I", _pick(r, [1280, 1500, 1000])) if typ == 2 else
                struct.pack("!I", r.randrange(40)) if typ == 4 else
                bytes(4) if r.random() < 0.8 else b"\x00\x09\x00\x01")
    else:
        typ = _pick(r, [3, 3, 3, 11, 11, 12, 5])
        code = {3: _pick(r, [0, 1, 3, 4, 13, 15, 16]), 11: _pick(r, [0, 1, 2]),
                12: _pick(r, [0, 1, 2, 3]), 5: _pick(r, [0, 1, 3, 4])}[typ]
        if typ == 5:
            rest = P.ip4(_pick(r, ["192.0.2.1", "224.0.0.5", "10.0.0.1"]))
        elif typ == 3 and code == 4:
            rest = struct.pack("!HH", 0, _pick(r, [1400, 0, 576]))
        elif typ == 12 and code == 0:
            rest = bytes([r.randrange(28), 0, 0, 0])
        else:
            rest = bytes(4)
        if r.random() < 0.2:  # RFC 4884 length / junk in the unused bytes
            rest = bytes([rest[0], r.randrange(1, 40)]) + rest[2:]
    pad = b"" if r.random() < 0.8 else bytes(r.randrange(1, 12))
    hdr = bytes([typ, code, 0, 0]) + rest
    # checksum as the reference validates it: header + embedded IP and
    # transport + rest, the embedded extension headers left out (icmp_any/
    # checksum.rs get_payload_for_checksum); sometimes left wrong on purpose
    covered = bytearray(emb + pad)
    for a, b in reversed(ext_ranges):
        del covered[a:b]
    msg = hdr + bytes(covered)
    if v6:
        ps = P.ip6(src) + P.ip6(dst) + struct.pack("!IxxxB", len(msg), 58)
        c = P.csum_fold(P.sum16(ps) + P.sum16(msg))
    else:
        c = P.csum_fold(P.sum16(msg))
    if r.random() < 0.1:
        c ^= 0x0101
    return hdr[:2] + struct.pack("!H", c) + hdr[4:] + emb + pad


def _l4_v4(r, proto, src, dst, payload):
    if proto == 1 and r.random() < 0.5:
        return _icmp_err(r, False, src, dst)
    sp, dp = _ports(r), _ports(r)
    if proto == 6:
        opts = b"" if r.random() < 0.7 else bytes([1] * (4 * r.randrange(1, 4)))
        return P.tcp(sp, dp, payload, P.pseudo4(src, dst, 6, 20 + len(opts) + len(payload)),
                     options=opts, reserved=r.choice([0, 0, 0, 0xE, 1]), flags=r.randrange(256))
    if proto == 17:
        return P.udp(sp, dp, payload, P.pseudo4(src, dst, 17, 8 + len(payload)))
    if proto == 1:
        typ = _pick(r, [0, 8, 8, 3, 11, 13, 14, 5, 42])
        rest = b"\x12\x34\x00\x01" if typ != 13 and typ != 14 else b"\x12\x34\x00\x01" + bytes(12)
        return P.icmp4(typ, 0, rest, payload)
    return payload


def _l4_v6(r, nh, src, dst, payload):
    if nh == 58 and r.random() < 0.5:
        return _icmp_err(r, True, src, dst)
    sp, dp = _ports(r), _ports(r)
    if nh == 6:
        return P.tcp(sp, dp, payload, P.pseudo6(src, dst, 6, 20 + len(payload)))
    if nh == 17:
        return P.udp(sp, dp, payload, P.pseudo6(src, dst, 17, 8 + len(payload)))
    if nh == 58:
        return P.icmp6(_pick(r, [128, 129, 1, 3, 135]), 0, b"\x00\x01\x00\x02", payload, src, dst)
    return payload


def _payload(r):
    k = r.random()
    if k < 0.5:
        n = r.randrange(0, 24)
    elif k < 0.9:
        n = r.randrange(24, 200)
    else:
        n = r.randrange(200, 1500)
    return bytes(r.randrange(256) for _ in range(min(n, 64))) + bytes(max(0, n - 64))


def _ip4_packet(r, src, dst, ttl=None):
    proto = _pick(r, [17, 17, 17, 6, 6, 1, 47, 51])
    pay = _payload(r)
    if proto == 51:  # IPv4 AH carrying UDP / TCP / something else
        inner = _pick(r, [17, 6, 1, 51, 47])
        body = _l4_v4(r, inner, src, dst, pay)
        body = P.ext_auth(inner, payload_len=_pick(r, [1, 1, 4, 0])) + body
    else:
        body = _l4_v4(r, proto, src, dst, pay)
    opts = b"" if r.random() < 0.85 else bytes([1] * (4 * r.randrange(1, 11)))
    ttl = ttl if ttl is not None else _pick(r, [64, 64, 64, 1, 2, 0, 255])
    ip = P.ipv4(src, dst, proto, len(body), ttl=ttl, options=opts, dscp=r.randrange(64),
                ecn=r.randrange(4), ident=r.randrange(65536), df=r.random() < 0.5,
                evil=r.random() < 0.1, mf=r.random() < 0.05)
    return ip + body, 0x0800


def _ip6_packet(r, src, dst):
    nh = _pick(r, [17, 17, 6, 58, 59])
    pay = _payload(r)
    body = _l4_v6(r, nh, src, dst, pay)
    # extension chain 0..5 long
    n_ext = _pick(r, [0, 0, 0, 1, 2, 3, 4, 5])
    chain = []
    for _ in range(n_ext):
        chain.append(_pick(r, [0, 43, 60, 44, 51]))
    for kind in reversed(chain):
        if kind == 44:
            body = P.ext_frag(nh, offset=r.randrange(4), more=r.random() < 0.3,
                              ident=r.randrange(1 << 32), reserved=r.randrange(2) * 0x5A,
                              res2=r.randrange(4))
        elif kind == 51:
            body = P.ext_auth(nh, payload_len=_pick(r, [1, 2, 4]), reserved=r.randrange(2) * 0x1234) + body
        else:
            body = P.ext_raw(nh, hdr_len=_pick(r, [0, 0, 1, 3]), fill=r.randrange(256)) + body if kind != 44 else body
        nh = kind
    ip = P.ipv6(src, dst, nh, len(body), hop=_pick(r, [64, 64, 1, 0, 2]), tc=r.randrange(256),
                flow=r.randrange(1 << 20))
    return ip + body, 0x86dd


def _vxlan_frame(r, inner_frame):
    """Outer IPv4/UDP/VXLAN to the local VTEP carrying ``inner_frame``."""
    vni = _pick(r, [1000, 1000, 1001, 1002, 2000, 999, 0, 1010, 1010, 1011])
    flags = 0x08 if r.random() < 0.9 else _pick(r, [0x00, 0x0C, 0x88])
    r1 = b"\0\0\0" if r.random() < 0.95 else b"\0\x01\0"
    vx = P.vxlan(vni, flags, r1, 0 if r.random() < 0.95 else 1)
    u = P.udp(r.randrange(49152, 65536), 4789 if r.random() < 0.95 else 4790, vx + inner_frame,
              csum=0 if r.random() < 0.7 else None,
              pseudo=P.pseudo4("100.65.0.2", VTEP4, 17, 8 + len(vx) + len(inner_frame)))
    ip = P.ipv4("100.65.0.2", VTEP4, 17, len(u), ttl=_pick(r, [64, 64, 1]), dscp=r.randrange(64),
                ecn=r.randrange(4))
    return P.l2(M1, PEER, 0x0800) + ip + u


def _inner_frame(r):
    if r.random() < 0.8:
        body, et = _ip4_packet(r, _pick(r, OVERLAY_V4_SRC), _pick(r, OVERLAY_V4_DST))
    else:
        body, et = _ip6_packet(r, _pick(r, OVERLAY_V6_SRC), _pick(r, OVERLAY_V6_DST))
    return P.l2("02:00:00:00:aa:01", "02:00:00:00:bb:01", et) + body


def _mutate(r, f: bytearray):
    k = r.random()
    if k < 0.10:                                   # truncate
        del f[r.randrange(0, len(f) + 1):]
    elif k < 0.25:                                 # flip bytes in the header region
        for _ in range(r.randrange(1, 4)):
            i = r.randrange(0, min(len(f), 90)) if len(f) else 0
            if i < len(f):
                f[i] = r.randrange(256)
    elif k < 0.28 and len(f) > 14:                 # ethertype games
        f[12:14] = _pick(r, [b"\x08\x06", b"\x88\xa8", b"\x91\x00", b"\x86\xdd", b"\x08\x00"])
    return f


def edge_frames(n: int, seed: int):
    """Returns a list of (frame, iif, flags, src_vni)."""
    r = random.Random(seed)
    out = []
    for _ in range(n):
        kind = r.random()
        iif, flags, svni = 1, 0, 0
        if kind < 0.30:                              # underlay v4 / v6
            if r.random() < 0.75:
                body, et = _ip4_packet(r, _pick(r, ["192.0.2.200", "198.51.100.2", "172.20.0.1",
                                                    "224.0.0.1", "255.255.255.255"] if r.random() < 0.1
                                                 else ["192.0.2.200", "10.9.9.9"]),
                                       _pick(r, UNDERLAY_V4))
            else:
                body, et = _ip6_packet(r, _pick(r, ["2001:db8:aa::1", "ff02::1"] if r.random() < 0.1
                                                else ["2001:db8:aa::1"]), _pick(r, UNDERLAY_V6))
            nv = _pick(r, [0, 0, 0, 0, 1, 2, 4, 5, 6])
            vl = [(_pick(r, [10, 20, 4094, 1]) if r.random() < 0.95 else _pick(r, [0, 4095]))
                  for _ in range(nv)]
            dmac = M1 if r.random() < 0.85 else _pick(r, ["ff:ff:ff:ff:ff:ff", "02:00:00:00:00:99",
                                                         "00:00:00:00:00:00", "01:00:5e:00:00:01"])
            smac = PEER if r.random() < 0.95 else _pick(r, ["00:00:00:00:00:00", "01:00:00:00:00:01"])
            f = P.l2(dmac, smac, et, vl) + body
            iif = 1 if r.random() < 0.8 else _pick(r, [2, 3, 4, 5, 6, 7, 8, 9, 10, 99])
            if iif != 1 and dmac == M1 and r.random() < 0.8:
                f = P.l2(f"02:00:00:00:00:{iif:02d}", smac, et, vl) + body
        elif kind < 0.50:                            # VXLAN to the VTEP (real decap)
            f = _vxlan_frame(r, _inner_frame(r))
        elif kind < 0.95:                            # seeded overlay (post-decap inner frame)
            f = _inner_frame(r)
            flags, svni = A.IN_SEEDED_OVERLAY, _pick(r, [1000, 1000, 1000, 1001, 1002, 2000, 999,
                                                         1010, 1010, 1010, 1011])
        else:                                        # non-IP / garbage
            f = P.l2(M1, PEER, _pick(r, [0x0806, 0x88cc, 0x8100])) + bytes(r.randrange(0, 60))
        f = bytearray(f)
        if r.random() < 0.35:
            f = _mutate(r, f)
        if r.random() < 0.15:                        # Ethernet padding / trailing bytes
            f += bytes(r.randrange(1, 20))
        out.append((bytes(f[:65535]), iif, flags, svni))
    # VPCs 1010 / 1011 (the fast overlay path): every NAT / PAT / ACL corner,
    # enumerated rather than left to the draw above
    for _ in range(600):
        src = _pick(r, FAST_V4_SRC)
        dst = _pick(r, FAST_V4_DST)
        proto = _pick(r, [6, 6, 17, 17, 1])
        pay = _payload(r)
        if proto == 1:
            body = _l4_v4(r, 1, src, dst, pay)
        else:
            sp, dp = _pick(r, FAST_PORTS), _pick(r, FAST_PORTS)
            body = (P.tcp(sp, dp, pay, P.pseudo4(src, dst, 6, 20 + len(pay))) if proto == 6 else
                    P.udp(sp, dp, pay, P.pseudo4(src, dst, 17, 8 + len(pay))))
        ip = P.ipv4(src, dst, proto, len(body), ttl=_pick(r, [64, 64, 64, 1]),
                    ident=r.randrange(65536))
        f = P.l2("02:00:00:00:aa:01", "02:00:00:00:bb:01", 0x0800) + ip + body
        out.append((f, 1, A.IN_SEEDED_OVERLAY, _pick(r, [1010, 1010, 1010, 1011])))
    return out


def pack_burst(frames, headroom: int = A.HEADROOM):
    """Lay frames out in one buffer (16-byte aligned slots, headroom in front)."""
    offs, total = [], 0
    for fr, *_ in frames:
        total += headroom
        offs.append(total)
        total = (total + len(fr) + 15) & ~15
    buf = np.zeros(total + 16, dtype=np.uint8)
    inp = np.zeros(len(frames), dtype=A.PKT_IN)
    for i, (fr, iif, flags, svni) in enumerate(frames):
        buf[offs[i]:offs[i] + len(fr)] = np.frombuffer(fr, dtype=np.uint8)
        inp[i] = (offs[i], len(fr), flags, iif, svni)
    return buf, inp
