"""TEST INFRASTRUCTURE: static-NAT configuration -> lowered NAT tables.

The reference turns VPC peerings and exposes into `NatTables` on the
management thread. Here that work is restated far enough to build the
reference's NAT known-answer tests -- address-only (NAT) and address + port
(PAT) -- from their own configurations:

- prefixes with optional port ranges and their set algebra:
  `PrefixWithPorts::{overlaps,subtract,merge}` `lpm/src/prefix/with_ports.rs:92-150`,
  `PortRange::{overlaps,subtract,merge,extend_right}` `:456-550`,
  `Prefix::{subtract,merge}` `lpm/src/prefix/mod.rs:298-430`
- exclusion collapse: `collapse_prefix_lists` `config/src/utils/collapse.rs:31-50`
- normalisation: `merge_overlapping_prefixes` / `merge_contiguous_prefixes`
  `config/src/utils/overlap.rs:67-134` (applied in `VpcExpose::validate`,
  `config/src/external/overlay/vpcpeering.rs:386-391`)
- `RangeBuilder` with ports: `nat/src/static_nat/setup/range_builder.rs:69-471`,
  `PortAddrTranslationValue::insert_and_merge` `nat/src/static_nat/setup/tables.rs:414-470`,
  `IpPortRange::extend_right` `nat/src/ranges.rs:55-70`, the Pat -> Nat
  conversion `tables.rs:550-590`
- `PerVniTable::add_peering` `nat/src/static_nat/setup/mod.rs:49-100`: one
  trie value per prefix, the last insert wins (`IpPrefixTrie::insert`)

Everything here is IPv4 (NAT44, `nat/src/lib.rs:19`).
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

Net = ipaddress.IPv4Network
MAXP = (0, 65535)


def P(s: str) -> Net:
    return ipaddress.ip_network(s, strict=True)


# ------------------------------------------------------------------ ports

def pr_len(p):
    return p[1] - p[0] + 1


def pr_overlaps(a, b):
    """PortRange::overlaps (with_ports.rs:458-462)."""
    return (a[0] <= b[0] <= a[1]) or (a[0] <= b[1] <= a[1]) or (b[0] <= a[0] and a[1] <= b[1])


def pr_intersection(a, b):
    if not pr_overlaps(a, b):
        return None
    return (max(a[0], b[0]), min(a[1], b[1]))


def pr_subtract(a, b):
    """PortRange::subtract (with_ports.rs:477-486)."""
    out = []
    if a[0] < b[0]:
        out.append((a[0], b[0] - 1))
    if a[1] > b[1]:
        out.append((b[1] + 1, a[1]))
    return out


def pr_merge(a, b):
    """PortRange::merge: overlapping or adjacent."""
    left, right = (a, b) if a[0] <= b[0] else (b, a)
    if left[1] + 1 < right[0]:
        return None
    return (left[0], max(left[1], right[1]))


# ------------------------------------------------------------------ prefixes

def covers(p: Net, q: Net) -> bool:
    return q.subnet_of(p)


def collides(p: Net, q: Net) -> bool:
    return covers(p, q) or covers(q, p)


def pfx_subtract(p: Net, other: Net) -> List[Net]:
    """Prefix::subtract (lpm/src/prefix/mod.rs:298-323)."""
    if not collides(p, other):
        return [p]
    if p.prefixlen >= other.prefixlen:
        return []
    out, cur = [], p
    for _ in range(other.prefixlen - p.prefixlen):
        lo, hi = cur.subnets(prefixlen_diff=1)
        if covers(lo, other):
            out.append(hi)
            cur = lo
        else:
            out.append(lo)
            cur = hi
    return out


def pfx_merge(p: Net, q: Net) -> Optional[Net]:
    """Prefix::merge (lpm/src/prefix/mod.rs:398-425)."""
    if covers(p, q):
        return p
    if covers(q, p):
        return q
    if p.prefixlen != q.prefixlen or p.prefixlen == 0:
        return None
    parent = p.supernet()
    return parent if covers(parent, q) else None


@dataclass(frozen=True)
class PP:
    """PrefixWithOptionalPorts: ports None means all ports (the constructor
    maps the full range to None, with_ports.rs:302-309)."""
    net: Net
    ports: Optional[Tuple[int, int]] = None

    @staticmethod
    def mk(net: Net, ports) -> "PP":
        return PP(net, None if ports is None or tuple(ports) == MAXP else tuple(ports))

    def p(self):
        return self.ports if self.ports is not None else MAXP

    def key(self):
        """Ord: (Ipv4Net (addr, len), Option<PortRange>) with None < Some."""
        return (int(self.net.network_address), self.net.prefixlen,
                0 if self.ports is None else 1, self.ports or (0, 0))

    def size(self) -> int:
        return self.net.num_addresses * pr_len(self.p())

    def overlaps(self, o: "PP") -> bool:
        return collides(self.net, o.net) and pr_overlaps(self.p(), o.p())

    def subtract(self, o: "PP") -> List["PP"]:
        """PrefixWithPorts::subtract (with_ports.rs:116-133)."""
        if not self.overlaps(o):
            return []
        out = [PP.mk(self.net, pr) for pr in pr_subtract(self.p(), o.p())]
        for q in pfx_subtract(self.net, o.net):
            i = pr_intersection(self.p(), o.p())
            if i is not None:
                out.append(PP.mk(q, i))
        return out

    def merge(self, o: "PP") -> Optional["PP"]:
        """PrefixWithPorts::merge (with_ports.rs:135-149)."""
        if self.net == o.net:
            m = pr_merge(self.p(), o.p())
            return None if m is None else PP.mk(self.net, m)
        if self.p() == o.p():
            m = pfx_merge(self.net, o.net)
            return None if m is None else PP.mk(m, self.p())
        return None


def ordered(s) -> List[PP]:
    return sorted(s, key=PP.key)


def collapse_prefix_lists(prefixes: List[PP], excludes: List[PP]) -> set:
    """collapse.rs:31-50: apply every exclusion to the (current) set."""
    result = set(prefixes)
    for ex in ordered(set(excludes)):
        for p in ordered(result):
            if p.overlaps(ex):
                result.remove(p)
                result.update(p.subtract(ex))
    return result


def merge_overlapping(prefixes: set) -> set:
    """overlap.rs:67-83."""
    todo = ordered(prefixes)
    merged = set()
    while todo:
        left = todo.pop()
        for right in todo:
            if left.overlaps(right):
                todo.extend(left.subtract(right))
                break
        else:
            merged.add(left)
    return merged


def merge_contiguous(prefixes: set) -> set:
    """overlap.rs:85-129 (stable sort by length, merge from the longest)."""
    uses_ports = did_merge = False
    merged = set()
    sp = sorted(ordered(prefixes), key=lambda p: p.net.prefixlen)
    while sp:
        left = sp.pop()
        if left.ports is not None:
            uses_ports = True
        for idx, right in enumerate(sp):
            m = left.merge(right)
            if m is not None:
                did_merge = True
                del sp[idx]
                ni = next((k for k, q in enumerate(sp) if q.net.prefixlen > m.net.prefixlen), len(sp))
                sp.insert(ni, m)
                break
        else:
            merged.add(left)
    if uses_ports and did_merge:
        return merge_contiguous(merged)
    return merged


def normalize(prefixes: set) -> List[PP]:
    return ordered(merge_contiguous(merge_overlapping(prefixes)))


def pp_list(items) -> List[PP]:
    """Exposes list prefixes as "a.b.c.d/n" or ("a.b.c.d/n", (lo, hi))."""
    out = []
    for it in items:
        if isinstance(it, str):
            out.append(PP.mk(P(it), None))
        else:
            out.append(PP.mk(P(it[0]), it[1]))
    return out


@dataclass
class Expose:
    ips: List
    nots: List = field(default_factory=list)
    as_range: List = field(default_factory=list)
    not_as: List = field(default_factory=list)
    nat: bool = True

    def ips_c(self) -> List[PP]:
        return normalize(collapse_prefix_lists(pp_list(self.ips), pp_list(self.nots)))

    def as_c(self) -> List[PP]:
        return normalize(collapse_prefix_lists(pp_list(self.as_range), pp_list(self.not_as)))


# ------------------------------------------------------------------ RangeBuilder

def add_offset(ip: int, port: int, ports, offset: int):
    """add_offset_to_address_and_port (range_builder.rs:69-107)."""
    n = pr_len(ports)
    covered, off_in = divmod(offset, n)
    if off_in > 65535 - port or port + off_in > ports[1]:
        covered += 1
    new_ip = ip + covered
    if new_ip > 0xFFFFFFFF:
        raise ValueError("MalformedPeering")
    return new_ip, ports[0] + ((port - ports[0]) + off_in) % n


def create_new_ranges(cur, end, tports):
    """create_new_ranges (range_builder.rs:325-424): (ip_lo, ip_hi, plo, phi)."""
    d = end[0] - cur[0]
    if d == 0:
        return [(cur[0], end[0], cur[1], end[1])]
    if d == 1:
        if cur[1] == tports[0] and end[1] == tports[1]:
            return [(cur[0], end[0], tports[0], tports[1])]
        return [(cur[0], cur[0], cur[1], tports[1]), (end[0], end[0], tports[0], end[1])]
    out = []
    smid, emid = cur, end
    if cur[1] != tports[0]:
        out.append((cur[0], cur[0], cur[1], tports[1]))
        smid = (cur[0] + 1, tports[0])
    if end[1] != tports[1]:
        emid = (end[0] - 1, tports[1])
    out.append((smid[0], emid[0], smid[1], emid[1]))
    if end[1] != tports[1]:
        out.append((end[0], end[0], tports[0], end[1]))
    return out


def rng_size(r):
    return (r[1] - r[0] + 1) * (r[3] - r[2] + 1)


class PatValue:
    """PortAddrTranslationValue: prefix port ranges + a map of disjoint
    ((ip, port) lo, (ip, port) hi) -> (IpPortRange, offset)."""

    def __init__(self, ports):
        self.ports = ports
        self.tree: Dict[tuple, list] = {}

    @staticmethod
    def _merge_bounds(left, right, ports):
        """merge_ip_port_range_bounds (tables.rs:440-470)."""
        (ls, le), (rs, re_) = left, right
        if le[0] == rs[0] and min(le[1] + 1, 65535) == rs[1]:
            return (ls, re_)
        if min(le[0] + 1, 0xFFFFFFFF) != rs[0] or le[1] != ports[1] or rs[1] != ports[0]:
            return None
        return (ls, re_)

    @staticmethod
    def _extend_right(a, b):
        """IpPortRange::extend_right (ranges.rs:55-70) on copies."""
        if (a[2], a[3]) == (b[2], b[3]):                 # same ports: IpRange::extend_right
            if a[0] > b[0] or a[1] >= b[0] or a[1] + 1 != b[0]:
                return None
            return (a[0], b[1], a[2], a[3])
        if (a[0], a[1]) == (b[0], b[1]):                 # same ips: PortRange::extend_right
            if a[2] > b[2] or a[3] >= b[2] or a[3] + 1 != b[2]:
                return None
            return (a[0], a[1], a[2], b[3])
        return None

    def insert_and_merge(self, key, value):
        self.tree[key] = value
        prev = [k for k in self.tree if k < key]
        if not prev:
            return
        pk = max(prev)
        mk = self._merge_bounds(pk, key, self.ports)
        if mk is None:
            return
        ext = self._extend_right(self.tree[pk][0], value[0])
        if ext is None:
            return
        off = self.tree[pk][1]
        self.tree[mk] = [ext, off]
        del self.tree[key]
        del self.tree[pk]


def range_builder(orig: List[PP], target: List[PP]):
    """RangeBuilder (range_builder.rs:133-303) with ports.  Yields
    (prefix, value); value is ("nat", [(olo, ohi, tlo, thi, off)], ip_len) or
    ("pat", ports, [(olo_ip, olo_port, ohi_ip, ohi_port, tlo, thi, tplo, tphi, off)], size)."""
    ti = 0
    tcur = None
    toff = 0
    if target:
        tcur = (int(target[0].net.network_address), target[0].p()[0])
    for op in orig:
        oports = op.p()
        value = PatValue(oports)
        osize = op.size()
        ocur = (int(op.net.network_address), oports[0])
        ooff = 0
        done = 0
        while done < osize:
            if ti >= len(target):
                raise ValueError("MalformedPeering: target space exhausted")
            tp = target[ti]
            trem = tp.size() - toff
            orem = osize - ooff
            size = orem if trem > orem else trem
            end = add_offset(tcur[0], tcur[1], tp.p(), size - 1)
            ranges = create_new_ranges(tcur, end, tp.p())
            c, off = ocur, ooff
            for k, r in enumerate(ranges):
                pe = add_offset(c[0], c[1], oports, rng_size(r) - 1)
                value.insert_and_merge((c, pe), [r, off])
                off += rng_size(r)
                if k != len(ranges) - 1:
                    c = add_offset(c[0], c[1], oports, rng_size(r))
            done += size
            if done < osize:
                ocur = add_offset(ocur[0], ocur[1], oports, size)
                ooff += size
            if size == trem:
                ti += 1
                toff = 0
                tcur = (int(target[ti].net.network_address), target[ti].p()[0]) \
                    if ti < len(target) else None
            else:
                tcur = add_offset(tcur[0], tcur[1], tp.p(), size)
                toff += size
        items = sorted(value.tree.items())
        as_nat = oports == MAXP and all(
            k[0][1] == 0 and k[1][1] == 65535 and (v[0][2], v[0][3]) == MAXP and v[1] % 65536 == 0
            for k, v in items)
        if as_nat:
            yield op.net, ("nat", [(k[0][0], k[1][0], v[0][0], v[0][1], v[1] // 65536)
                                   for k, v in items],
                           sum(v[0][1] - v[0][0] + 1 for _, v in items))
        else:
            yield op.net, ("pat", oports,
                           [(k[0][0], k[0][1], k[1][0], k[1][1], v[0][0], v[0][1], v[0][2], v[0][3],
                             v[1]) for k, v in items],
                           sum(rng_size(v[0]) for _, v in items))


@dataclass
class Peering:
    """One direction of a peering as seen from `local_vni`."""
    local_vni: int
    remote_vni: int
    local: List[Expose]
    remote: List[Expose]


def nat_tables(peerings: List[Peering]):
    """PerVniTable per local VNI: src_nat[dst_vni] from the local NAT exposes
    (private -> public), dst_nat from the remote NAT exposes (public ->
    private).  Returns {(kind, src_vni, dst_vni): {prefix: value}}; a prefix
    inserted twice keeps the last value (IpPrefixTrie::insert)."""
    out: Dict[Tuple[int, int, int], Dict[Net, tuple]] = {}
    for pr in peerings:
        for e in pr.local:
            if not e.nat or not e.as_range:
                continue
            tab = out.setdefault((1, pr.local_vni, pr.remote_vni), {})
            for pfx, val in range_builder(e.ips_c(), e.as_c()):
                tab[pfx] = val
        dtab = out.setdefault((0, pr.local_vni, 0), {})
        for e in pr.remote:
            if not e.nat or not e.as_range:
                continue
            for pfx, val in range_builder(e.as_c(), e.ips_c()):
                dtab[pfx] = val
    return out


def _ip(x: int) -> str:
    return str(ipaddress.IPv4Address(x))


def lower(tb, tables) -> None:
    """Add the tables to a dataplane_amd.tables.TablesBuilder."""
    for (kind, svni, dvni), entries in sorted(tables.items()):
        ents = []
        for pfx, val in sorted(entries.items(), key=lambda kv: (int(kv[0].network_address),
                                                               kv[0].prefixlen)):
            if val[0] == "nat":
                ents.append(dict(prefix=str(pfx), size=val[2], ranges=[
                    (_ip(olo), 0, _ip(ohi), 65535, _ip(tlo), _ip(thi), 0, 65535, off)
                    for (olo, ohi, tlo, thi, off) in val[1]]))
            else:
                ents.append(dict(prefix=str(pfx), pat=True, port_ranges=[val[1]], size=val[3],
                                 ranges=[(_ip(a), ap, _ip(b), bp, _ip(c), _ip(d), cp, dp, off)
                                         for (a, ap, b, bp, c, d, cp, dp, off) in val[2]]))
        tb.add_nat_table(kind, svni, dvni, ents)
