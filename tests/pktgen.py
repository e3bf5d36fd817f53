"""Frame builder for the parity tests: Ethernet / 802.1Q / IPv4 (+options) /
IPv6 (+extension headers) / UDP / TCP / ICMP / VXLAN, with every field
overridable so malformed frames can be written on purpose."""
from __future__ import annotations

import ipaddress
import struct


def csum_fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def sum16(b: bytes) -> int:
    if len(b) & 1:
        b = b + b"\0"
    return sum(struct.unpack(f"!{len(b) // 2}H", b))


def mac(s) -> bytes:
    if isinstance(s, (bytes, bytearray)):
        return bytes(s)
    return bytes(int(x, 16) for x in s.split(":"))


def ip4(a) -> bytes:
    return ipaddress.IPv4Address(a).packed if not isinstance(a, bytes) else a


def ip6(a) -> bytes:
    return ipaddress.IPv6Address(a).packed if not isinstance(a, bytes) else a


def eth(dst, src, ethertype: int) -> bytes:
    return mac(dst) + mac(src) + struct.pack("!H", ethertype)


def vlan(vid: int, ethertype: int, pcp: int = 0, dei: int = 0) -> bytes:
    return struct.pack("!HH", (pcp << 13) | (dei << 12) | (vid & 0xFFF), ethertype)


def ipv4(src, dst, proto: int, payload_len: int, ttl: int = 64, options: bytes = b"",
         dscp: int = 0, ecn: int = 0, ident: int = 0, df: bool = True, mf: bool = False,
         evil: bool = False, frag_off: int = 0, version: int = 4, ihl: int | None = None,
         total_len: int | None = None, csum: int | None = None) -> bytes:
    hl = 20 + len(options)
    ihl = hl // 4 if ihl is None else ihl
    tl = hl + payload_len if total_len is None else total_len
    fl = (int(evil) << 15) | (int(df) << 14) | (int(mf) << 13) | (frag_off & 0x1FFF)
    h = struct.pack("!BBHHHBBH4s4s", (version << 4) | (ihl & 0xF), (dscp << 2) | ecn,
                    tl & 0xFFFF, ident, fl, ttl, proto, 0, ip4(src), ip4(dst)) + options
    c = csum_fold(sum16(h)) if csum is None else csum
    return h[:10] + struct.pack("!H", c) + h[12:]


def ipv6(src, dst, nh: int, payload_len: int, hop: int = 64, tc: int = 0, flow: int = 0,
         plen: int | None = None) -> bytes:
    pl = payload_len if plen is None else plen
    return struct.pack("!IHBB16s16s", (6 << 28) | (tc << 20) | (flow & 0xFFFFF), pl & 0xFFFF,
                       nh, hop, ip6(src), ip6(dst))


def ext_raw(nh: int, hdr_len: int = 0, fill: int = 0) -> bytes:
    """Hop-by-hop / routing / destination options: (len+1)*8 bytes."""
    n = (hdr_len + 1) * 8
    return bytes([nh, hdr_len]) + bytes([fill]) * (n - 2)


def ext_frag(nh: int, offset: int = 0, more: bool = False, ident: int = 0,
             reserved: int = 0, res2: int = 0) -> bytes:
    return struct.pack("!BBHI", nh, reserved, (offset << 3) | (res2 << 1) | int(more), ident)


def ext_auth(nh: int, payload_len: int = 1, spi: int = 0x100, seq: int = 1,
             reserved: int = 0) -> bytes:
    n = (payload_len + 2) * 4
    icv = bytes(range(max(0, n - 12)))
    return struct.pack("!BBHII", nh, payload_len, reserved, spi, seq) + icv[:max(0, n - 12)]


def udp(sport: int, dport: int, payload: bytes, pseudo: bytes | None = None,
        length: int | None = None, csum: int | None = None) -> bytes:
    ln = 8 + len(payload) if length is None else length
    h = struct.pack("!HHHH", sport, dport, ln & 0xFFFF, 0)
    if csum is None:
        if pseudo is None:
            csum = 0
        else:
            c = csum_fold(sum16(pseudo) + sum16(h + payload))
            csum = 0xFFFF if c == 0 else c
    return h[:6] + struct.pack("!H", csum) + payload


def tcp(sport: int, dport: int, payload: bytes, pseudo: bytes | None = None, seq: int = 1,
        ack: int = 0, flags: int = 0x18, window: int = 4096, options: bytes = b"",
        doff: int | None = None, reserved: int = 0, urg: int = 0,
        csum: int | None = None) -> bytes:
    d = (20 + len(options)) // 4 if doff is None else doff
    h = struct.pack("!HHIIBBHHH", sport, dport, seq, ack, (d << 4) | (reserved & 0xF),
                    flags & 0xFF, window, 0, urg) + options
    if csum is None:
        csum = csum_fold(sum16(pseudo) + sum16(h + payload)) if pseudo is not None else 0
    return h[:16] + struct.pack("!H", csum) + h[18:] + payload


def icmp4(typ: int, code: int, rest: bytes, payload: bytes = b"") -> bytes:
    h = bytes([typ, code, 0, 0]) + rest
    c = csum_fold(sum16(h + payload))
    return h[:2] + struct.pack("!H", c) + h[4:] + payload


def icmp6(typ: int, code: int, rest: bytes, payload: bytes, src, dst) -> bytes:
    body = bytes([typ, code, 0, 0]) + rest + payload
    ps = ip6(src) + ip6(dst) + struct.pack("!IxxxB", len(body), 58)
    c = csum_fold(sum16(ps) + sum16(body))
    return body[:2] + struct.pack("!H", c) + body[4:]


def vxlan(vni: int, flags: int = 0x08, r1: bytes = b"\0\0\0", r2: int = 0) -> bytes:
    return bytes([flags]) + r1 + struct.pack("!I", (vni << 8) | r2)


def pseudo4(src, dst, proto: int, length: int) -> bytes:
    return ip4(src) + ip4(dst) + struct.pack("!BBH", 0, proto, length)


def pseudo6(src, dst, nh: int, length: int) -> bytes:
    return ip6(src) + ip6(dst) + struct.pack("!IxxxB", length, nh)


def l4(proto: int, sport: int, dport: int, payload: bytes, pseudo: bytes | None, **kw) -> bytes:
    if proto == 6:
        return tcp(sport, dport, payload, pseudo, **kw)
    if proto == 17:
        return udp(sport, dport, payload, pseudo, **kw)
    return payload


def udp4_frame(dmac, smac, src, dst, sport=1234, dport=5678, payload=b"\0" * 18, ttl=64,
               vlans=(), **ipkw) -> bytes:
    u = udp(sport, dport, payload, pseudo4(src, dst, 17, 8 + len(payload)))
    return l2(dmac, smac, 0x0800, vlans) + ipv4(src, dst, 17, len(u), ttl=ttl, **ipkw) + u


def l2(dmac, smac, ethertype: int, vlans=()) -> bytes:
    if not vlans:
        return eth(dmac, smac, ethertype)
    out = eth(dmac, smac, 0x8100)
    for k, vid in enumerate(vlans):
        out += vlan(vid, 0x8100 if k + 1 < len(vlans) else ethertype)
    return out
