"""CPU: v6 address lookups of one site against the oracle -- the kernel body
on the host (tests/emu).

- The classifiers' v6 address index (dp_tables.cpp build_field_index:
  sorted bounds narrowed by a 16-bit jump table), for rule sets whose shared
  prefix is /48, /32, /8 or none, with addresses inside the rules, between
  them, at the site's edges and outside it on both sides, in both classifier
  forms.
- The v6 FIB's window table (Lpm.wtab, dp_tables.cpp add_v6_window): routes of
  one site, a shorter route covering it and the /0, looked up from inside the
  site, at its edges and outside it."""
import ipaddress
import random
import zlib

import pytest

from dataplane_amd import _abi as A
from dataplane_amd.tables import ALLOW, DENY, TablesBuilder as TB
from edgecase import pack_burst
from golden.kat import IF_MAC, NH_MAC, OIF_MAC, PEER_MAC
from helpers import compare, hist
from oracle.pyoracle import Oracle
import pktgen as P
import pyemu

VNI_A, VNI_B = 2000, 3000


def tables(rule_nets, r: random.Random):
    t = TB(genid=1)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    nh = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh)
    for v in (VNI_A, VNI_B):
        f = t.add_fib(v, vnis=[v])
        t.add_route(f, "0.0.0.0/0", nh)
        t.add_route(f, "::/0", nh)
    t.add_ff_remote(VNI_A, "::/0", VNI_B)
    t.add_ff_local(VNI_A, VNI_B, "::/0")
    t.add_acl_default(VNI_A, VNI_B, DENY)
    for k, (s, d) in enumerate(rule_nets):
        t.add_acl(VNI_A, VNI_B, ALLOW if k % 3 else DENY, family=6,
                  src=s, dst=d, dports=(0, 65535) if k % 4 else (1000 + k, 1000 + k))
    return t


def addr_in(net: str, r: random.Random) -> str:
    n = ipaddress.ip_network(net)
    return str(n.network_address + r.randrange(n.num_addresses))


def probes(rule_nets, site: str, r: random.Random):
    """Addresses inside rules, inside the site but outside rules, at the
    site's first and last address and just beyond them, and far outside."""
    n = ipaddress.ip_network(site)
    first, last = int(n.network_address), int(n.broadcast_address)
    out = []
    for s, d in rule_nets:
        out += [addr_in(s, r), addr_in(d, r)]
        for net in (s, d):
            m = ipaddress.ip_network(net)
            out += [str(m.network_address), str(m.broadcast_address)]
            if int(m.broadcast_address) < (1 << 128) - 1:
                out.append(str(ipaddress.IPv6Address(int(m.broadcast_address) + 1)))
    out += [addr_in(site, r) for _ in range(40)]
    for x in (first, last, first - 1, last + 1, 0, 1, (1 << 128) - 1, first >> 1, (last + 1) << 1):
        if 0 <= x < (1 << 128):
            out.append(str(ipaddress.IPv6Address(x)))
    return out


@pytest.mark.parametrize("site,plen", [("2001:db8:1::/48", 64), ("2001:db8::/32", 56),
                                       ("2000::/8", 40), ("::/0", 24)])
@pytest.mark.parametrize("form", ["list", "bv"])
def test_v6_window_index(site, plen, form, cls_form):
    r = random.Random(zlib.crc32(f"{site}/{plen}".encode()))
    n = ipaddress.ip_network(site)
    rule_nets = []
    for k in range(60):
        a = n.network_address + r.randrange(n.num_addresses)
        b = n.network_address + r.randrange(n.num_addresses)
        rule_nets.append((str(ipaddress.ip_network(f"{a}/{plen + r.randrange(12)}", strict=False)),
                          str(ipaddress.ip_network(f"{b}/{plen + r.randrange(12)}", strict=False))))
    # rules touching the site's last address (their end is the site's end)
    last = ipaddress.ip_network(site).broadcast_address
    rule_nets.append((str(ipaddress.ip_network(f"{last}/{plen}", strict=False)), "::/0"))
    t = tables(rule_nets, r)
    cls_form(pyemu.lib(), form)
    addrs = probes(rule_nets, site, r)
    frames = []
    for k in range(3000):
        if k % 2:
            s, d = r.choice(rule_nets)  # inside one rule's prefixes (its ports may not match)
            src, dst = addr_in(s, r), addr_in(d, r)
        else:
            src, dst = r.choice(addrs), r.choice(addrs)
        body = P.udp(r.randrange(1, 65535), r.choice([80, 1000 + r.randrange(61), 4000]), b"x" * 8,
                     P.pseudo6(src, dst, 17, 16))
        fr = P.eth(IF_MAC, PEER_MAC, 0x86DD) + P.ipv6(src, dst, 17, len(body)) + body
        frames.append((fr, 1, A.IN_SEEDED_OVERLAY, VNI_A))
    buf, inp = pack_burst(frames)
    tp = t.build()
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = pyemu.process(tp, b_dut, inp)
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"v6 window {site} {form}")
    h = hist(o_ref)
    assert h.get("Delivered", 0) > 100 and h.get("AclDropped", 0) > 100, h


@pytest.mark.parametrize("site,lens", [("2001:db8::/32", (32, 64)), ("2001:db8:77::/48", (48, 90)),
                                       ("fd00::/24", (24, 40))])
def test_v6_fib_window(site, lens):
    """The v6 FIB's window table (Lpm.wtab): routes of one site, a shorter
    route covering the site and the /0, looked up from inside the site, at its
    edges and outside it; each route its own FibEntry, so the packet's
    metadata names the route that matched."""
    r = random.Random(zlib.crc32(str(site).encode()))
    t = TB(genid=1)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    nhs = []
    for k in range(12):
        t.add_adjacency(f"192.0.2.{k + 1}", 10, NH_MAC)
        nhs.append(t.add_nh([[TB.egress(10, f"192.0.2.{k + 1}")]]))
    t.add_route(t.add_fib(0), "0.0.0.0/0", nhs[0])
    for v in (VNI_A, VNI_B):
        f = t.add_fib(v, vnis=[v])
        t.add_route(f, "0.0.0.0/0", nhs[0])
        if v == VNI_B:
            n = ipaddress.ip_network(site)
            t.add_route(f, "::/0", nhs[1])
            t.add_route(f, str(n.supernet(new_prefix=max(0, n.prefixlen - 4))), nhs[2])
            nets = []
            for k in range(400):
                a = n.network_address + r.randrange(n.num_addresses)
                nets.append(str(ipaddress.ip_network(f"{a}/{r.randrange(lens[0], lens[1] + 1)}", strict=False)))
                t.add_route(f, nets[-1], nhs[3 + k % 9])
        else:
            t.add_route(f, "::/0", nhs[0])
    t.add_ff_remote(VNI_A, "::/0", VNI_B)
    t.add_ff_local(VNI_A, VNI_B, "::/0")
    n = ipaddress.ip_network(site)
    first, last = int(n.network_address), int(n.broadcast_address)
    dsts = [addr_in(x, r) for x in nets] + [addr_in(site, r) for _ in range(200)]
    for x in (first, last, first - 1, last + 1, 0, (1 << 128) - 1, first - (1 << 100), last + (1 << 100)):
        if 0 <= x < (1 << 128):
            dsts.append(str(ipaddress.IPv6Address(x)))
    frames = []
    for k in range(3000):
        dst = r.choice(dsts)
        src = "2001:db8:ffff::1"
        body = P.udp(1234, 80, b"x" * 8, P.pseudo6(src, dst, 17, 16))
        fr = P.eth(IF_MAC, PEER_MAC, 0x86DD) + P.ipv6(src, dst, 17, len(body)) + body
        frames.append((fr, 1, A.IN_SEEDED_OVERLAY, VNI_A))
    buf, inp = pack_burst(frames)
    tp = t.build()
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = pyemu.process(tp, b_dut, inp)
    compare(o_ref, b_ref, o_dut, b_dut, inp, f"v6 FIB window {site}")
    assert len(set(o_ref["fib_entry"].tolist())) >= 10  # many routes, the covering one and the /0 hit


def test_v6_window_budget():
    """Window tables stay within a budget over the image (dp_tables.cpp
    build_image v6wtb): 100 VPC FIBs, each with one /40 route, would need
    100 x 4 MiB of 20-bit windows; they get 16-bit ones instead, and lookups
    through them still match the oracle."""
    r = random.Random(7)
    t = TB(genid=1)
    t.add_iface(1, IF_MAC)
    t.add_iface(10, OIF_MAC)
    t.add_adjacency("192.0.2.1", 10, NH_MAC)
    t.add_adjacency("192.0.2.2", 10, NH_MAC)
    nh0 = t.add_nh([[TB.egress(10, "192.0.2.1")]])
    nh1 = t.add_nh([[TB.egress(10, "192.0.2.2")]])
    t.add_route(t.add_fib(0), "0.0.0.0/0", nh0)
    vnis = [5000 + k for k in range(100)]
    for k, v in enumerate(vnis):
        f = t.add_fib(v, vnis=[v])
        t.add_route(f, "0.0.0.0/0", nh0)
        t.add_route(f, "::/0", nh0)
        t.add_route(f, f"2001:db8:{k:x}00::/40", nh1)
    t.add_ff_remote(VNI_A, "::/0", vnis[3])
    t.add_ff_local(VNI_A, vnis[3], "::/0")
    t.add_fib(VNI_A, vnis=[VNI_A])
    tp = t.build()
    assert pyemu.lib().dpemu_image_bytes(tp) < (128 << 20)
    frames = []
    for k in range(400):
        dst = f"2001:db8:{3 if k % 2 else 4:x}{r.randrange(256):02x}::{r.randrange(1, 65535):x}"
        src = "2001:db8:ffff::1"
        body = P.udp(1234, 80, b"x" * 8, P.pseudo6(src, dst, 17, 16))
        fr = P.eth(IF_MAC, PEER_MAC, 0x86DD) + P.ipv6(src, dst, 17, len(body)) + body
        frames.append((fr, 1, A.IN_SEEDED_OVERLAY, VNI_A))
    buf, inp = pack_burst(frames)
    b_ref, b_dut = buf.copy(), buf.copy()
    o_ref = Oracle(tp).process(b_ref, inp)
    o_dut = pyemu.process(tp, b_dut, inp)
    compare(o_ref, b_ref, o_dut, b_dut, inp, "v6 window budget")
    assert len(set(o_ref["fib_entry"].tolist())) == 2
