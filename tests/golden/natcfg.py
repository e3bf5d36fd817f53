"""TEST INFRASTRUCTURE: static-NAT configuration -> lowered NAT tables.

The reference turns VPC peerings and exposes into `NatTables` on the
management thread. Here that work is restated just far enough to build the
reference's NAT known-answer tests from their own configurations:

- `ip` / `not` and `as_range` / `not_as` exclusion collapse:
  `config/src/utils/collapse.rs:7-50`, `Prefix::subtract`
  `lpm/src/prefix/mod.rs:298-323`, `normalize` `config/src/utils/overlap.rs:132`
- `RangeBuilder` without port ranges: `nat/src/static_nat/setup/range_builder.rs:119-301`
- `PerVniTable::add_peering`: `nat/src/static_nat/setup/mod.rs:49-100`

Only the address-only (NAT, not PAT) case is restated; the tests that use it
are the address-translation KATs of `nat/src/static_nat/test.rs`.
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

Net = ipaddress.IPv4Network


def P(s: str) -> Net:
    return ipaddress.ip_network(s, strict=True)


def subtract(p: Net, other: Net) -> List[Net]:
    """Prefix::subtract: split `p` around `other`, emitting the halves that
    do not contain it (lpm/src/prefix/mod.rs:298-323)."""
    if not p.overlaps(other):
        return [p]
    if p.prefixlen >= other.prefixlen:
        return []
    out, cur = [], p
    for _ in range(other.prefixlen - p.prefixlen):
        lo, hi = cur.subnets(prefixlen_diff=1)
        if other.subnet_of(lo):
            out.append(hi)
            cur = lo
        else:
            out.append(lo)
            cur = hi
    return out


def collapse(prefixes: List[Net], excludes: List[Net]) -> List[Net]:
    """collapse_prefix_lists + normalize: apply exclusions, then merge
    overlapping / contiguous prefixes; result sorted by address."""
    res = set(prefixes)
    for ex in excludes:
        for p in list(res):
            if p.overlaps(ex):
                res.remove(p)
                res.update(subtract(p, ex))
    return sorted(ipaddress.collapse_addresses(res), key=lambda n: (int(n.network_address),
                                                                    n.prefixlen))


@dataclass
class Expose:
    ips: List[str]
    nots: List[str] = field(default_factory=list)
    as_range: List[str] = field(default_factory=list)
    not_as: List[str] = field(default_factory=list)
    nat: bool = True

    def ips_c(self) -> List[Net]:
        return collapse([P(x) for x in self.ips], [P(x) for x in self.nots])

    def as_c(self) -> List[Net]:
        return collapse([P(x) for x in self.as_range], [P(x) for x in self.not_as])


def range_builder(orig: List[Net], target: List[Net]):
    """RangeBuilder (address-only): walk a virtual flat list of the target
    prefixes; each original prefix takes the next `size` addresses, possibly
    spanning several target prefixes.  Yields (prefix, ranges) with ranges
    (orig_lo, orig_hi, tgt_lo, tgt_hi, offset_in_orig_prefix)."""
    ti, toff = 0, 0
    for p in orig:
        size = p.num_addresses
        done, ranges = 0, []
        while done < size:
            if ti >= len(target):
                raise ValueError("MalformedPeering: target space exhausted")
            t = target[ti]
            take = min(t.num_addresses - toff, size - done)
            olo = int(p.network_address) + done
            tlo = int(t.network_address) + toff
            ranges.append((olo, olo + take - 1, tlo, tlo + take - 1, done))
            done += take
            toff += take
            if toff == t.num_addresses:
                ti, toff = ti + 1, 0
        yield p, ranges


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
    private).  Returns {(kind, src_vni, dst_vni): {prefix: ranges}}."""
    out: Dict[Tuple[int, int, int], Dict[Net, list]] = {}
    for pr in peerings:
        for e in pr.local:
            if not e.nat or not e.as_range:
                continue
            tab = out.setdefault((1, pr.local_vni, pr.remote_vni), {})
            for pfx, rg in range_builder(e.ips_c(), e.as_c()):
                tab[pfx] = rg
        dtab = out.setdefault((0, pr.local_vni, 0), {})
        for e in pr.remote:
            if not e.nat or not e.as_range:
                continue
            for pfx, rg in range_builder(e.as_c(), e.ips_c()):
                dtab[pfx] = rg
    return out


def lower(tb, tables) -> None:
    """Add the tables to a dataplane_amd.tables.TablesBuilder."""
    for (kind, svni, dvni), entries in sorted(tables.items()):
        ents = []
        for pfx, ranges in sorted(entries.items(), key=lambda kv: (int(kv[0].network_address),
                                                                   kv[0].prefixlen)):
            ents.append(dict(prefix=str(pfx), size=pfx.num_addresses, ranges=[
                (str(ipaddress.IPv4Address(olo)), 0, str(ipaddress.IPv4Address(ohi)), 65535,
                 str(ipaddress.IPv4Address(tlo)), str(ipaddress.IPv4Address(thi)), 0, 65535, off)
                for (olo, ohi, tlo, thi, off) in ranges]))
        tb.add_nat_table(kind, svni, dvni, ents)
