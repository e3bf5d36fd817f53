# SPDX-License-Identifier: Apache-2.0
"""Python builder for the lowered table descriptors (``dp_tables_desc_t``).

This is what a host integration does before ``dp_tables_publish``: lower the
reference's structures (FIB routes / FibEntry instructions, interface and
adjacency tables, ACL and flow-filter rules, static NAT tables) into flat
arrays.  Used by the tests (known-answer tables) and by examples.
"""
from __future__ import annotations

import ctypes as C
import ipaddress
from typing import List, Optional, Sequence, Tuple

from . import _abi as A

INSTR_DROP, INSTR_LOCAL, INSTR_ENCAP, INSTR_EGRESS = 0, 1, 2, 3
IF_UNKNOWN, IF_DOWN, IF_UP = 0, 1, 2
IFT_UNKNOWN, IFT_ETHERNET, IFT_DOT1Q, IFT_LOOPBACK, IFT_VXLAN = 0, 1, 2, 3, 4
ATTACH_NONE, ATTACH_VRF, ATTACH_BRIDGE = 0, 1, 2
NAT_NONE, NAT_STATIC, NAT_MASQUERADE, NAT_PORT_FORWARDING = 0, 1, 2, 3
ALLOW, DENY = 0, 1


def mac_bytes(m) -> bytes:
    if isinstance(m, (bytes, bytearray)):
        return bytes(m)
    return bytes(int(x, 16) for x in m.split(":"))


def ip_obj(a):
    return ipaddress.ip_address(a) if not isinstance(a, (ipaddress.IPv4Address,
                                                         ipaddress.IPv6Address)) else a


def mk_ip(a) -> A.IpAddr:
    r = A.IpAddr()
    if a is None:
        return r
    a = ip_obj(a)
    r.family = 4 if a.version == 4 else 6
    b = a.packed
    for i, x in enumerate(b):
        r.addr[i] = x
    return r


def mk_prefix(p) -> A.Prefix:
    n = ipaddress.ip_network(p, strict=True)
    r = A.Prefix()
    r.family = 4 if n.version == 4 else 6
    r.len = n.prefixlen
    for i, x in enumerate(n.network_address.packed):
        r.addr[i] = x
    return r


def wildcard(family: int) -> A.Prefix:
    return mk_prefix("0.0.0.0/0" if family == 4 else "::/0")


class TablesBuilder:
    def __init__(self, genid: int = 1):
        self.genid = genid
        self.fibs: List[A.Fib] = []
        self.vnis: List[A.VniFib] = []
        self.routes: List[A.Route] = []
        self.nhs: List[A.RouteNh] = []
        self.entries: List[A.FibEntry] = []
        self.instrs: List[A.Instr] = []
        self.ifaces: List[A.Iface] = []
        self.adjs: List[A.Adjacency] = []
        self.acl = {4: [], 6: []}
        self.acl_defaults: List[A.AclDefault] = []
        self.ff_remote = {4: [], 6: []}
        self.ff_local = {4: [], 6: []}
        self.nat_tables: List[A.NatTable] = []
        self.nat_entries: List[A.NatEntry] = []
        self.nat_prs: List[A.PortRange] = []
        self.nat_ranges: List[A.NatRange] = []
        self.portfw: List[A.PortFwRule] = []
        self.masq: List[A.MasqExpose] = []
        self.masq_prefixes: List[A.Prefix] = []
        self.masq_claims: List[A.MasqClaim] = []
        self.masq_config_tag = 0
        # MasqueradeConfig::set_randomize (dpgpu.h dp_masq_expose_t): the port
        # blocks of each address in a permuted order drawn from masq_seed
        self.masq_randomize = False
        self.masq_seed = 0
        self._keep = []

    # -- routing --------------------------------------------------------------
    def add_fib(self, vrf_id: int, vtep_ip=None, vtep_mac=None, vnis: Sequence[int] = ()) -> int:
        f = A.Fib()
        f.vrf_id = vrf_id
        if vtep_ip is not None:
            f.flags |= 1
            f.vtep_ip = mk_ip(vtep_ip)
        if vtep_mac is not None:
            f.flags |= 2
            for i, x in enumerate(mac_bytes(vtep_mac)):
                f.vtep_mac[i] = x
        self.fibs.append(f)
        idx = len(self.fibs) - 1
        for v in vnis:
            self.vnis.append(A.VniFib(v, idx))
        return idx

    @staticmethod
    def drop() -> A.Instr:
        return A.Instr(kind=INSTR_DROP)

    @staticmethod
    def local(ifindex: int = 0) -> A.Instr:
        return A.Instr(kind=INSTR_LOCAL, ifindex=ifindex)

    @staticmethod
    def egress(ifindex: Optional[int], addr=None) -> A.Instr:
        i = A.Instr(kind=INSTR_EGRESS)
        if ifindex is not None:
            i.flags |= 1
            i.ifindex = ifindex
        if addr is not None:
            i.flags |= 2
            i.addr = mk_ip(addr)
        return i

    @staticmethod
    def encap(vni: int, remote, dmac=None) -> A.Instr:
        i = A.Instr(kind=INSTR_ENCAP, vni=vni)
        i.addr = mk_ip(remote)
        if dmac is not None:
            i.flags |= 4
            for k, x in enumerate(mac_bytes(dmac)):
                i.mac[k] = x
        return i

    def add_nh(self, entries: Sequence[Sequence[A.Instr]]) -> int:
        """A FibRoute: one or more FibEntries (ECMP), each an instruction list."""
        first = len(self.entries)
        for ins in entries:
            self.entries.append(A.FibEntry(len(self.instrs), len(ins)))
            self.instrs.extend(ins)
        self.nhs.append(A.RouteNh(first, len(entries)))
        return len(self.nhs) - 1

    def add_route(self, fib: int, prefix: str, nh: int) -> None:
        self.routes.append(A.Route(mk_prefix(prefix), fib, nh))

    def add_iface(self, ifindex: int, mac, admin=IF_UP, oper=IF_UP, iftype=IFT_ETHERNET,
                  attach=ATTACH_VRF, vrf_id: int = 0) -> None:
        i = A.Iface(ifindex=ifindex, admin_state=admin, oper_state=oper, iftype=iftype,
                    attach=attach, vrf_id=vrf_id)
        for k, x in enumerate(mac_bytes(mac)):
            i.mac[k] = x
        self.ifaces.append(i)

    def add_adjacency(self, addr, ifindex: int, mac) -> None:
        a = A.Adjacency(addr=mk_ip(addr), ifindex=ifindex)
        for k, x in enumerate(mac_bytes(mac)):
            a.mac[k] = x
        self.adjs.append(a)

    # -- classifiers ------------------------------------------------------------
    @staticmethod
    def rule(family: int, proto: Optional[int] = None, vni_a: int = 0, vni_b: int = 0,
             gate: int = 0, src: Optional[str] = None, dst: Optional[str] = None,
             sports: Tuple[int, int] = (0, 65535), dports: Tuple[int, int] = (0, 65535),
             priority: int = 0, action: int = 0, action2: int = 0) -> A.Rule:
        r = A.Rule(family=family, gate=gate, vni_a=vni_a, vni_b=vni_b, priority=priority,
                   action=action, action2=action2)
        if proto is not None:
            r.proto_val, r.proto_mask = proto, 0xFF
        r.sport_lo, r.sport_hi = sports
        r.dport_lo, r.dport_hi = dports
        r.src = mk_prefix(src) if src else wildcard(family)
        r.dst = mk_prefix(dst) if dst else wildcard(family)
        return r

    def add_acl(self, src_vni: int, dst_vni: int, action: int, family: int = 4,
                scope: int = A.ACL_SCOPE_FLOW, **kw) -> None:
        """ACL rules are matched in insertion order (first match); `scope` is
        AclScope (Flow by default, config/src/external/overlay/acl.rs:137-141)."""
        self.acl[family].append(self.rule(family, vni_a=src_vni, vni_b=dst_vni, action=action,
                                          action2=scope, **kw))

    def add_acl_default(self, src_vni: int, dst_vni: int, action: int) -> None:
        self.acl_defaults.append(A.AclDefault(src_vni, dst_vni, action))

    def add_ff_remote(self, src_vni: int, dst_prefix: str, dst_vni: int, dst_nat: int = NAT_NONE,
                      proto: Optional[int] = None, dports=(0, 65535), gate_vni: int = 0,
                      port_forwarding: bool = False) -> None:
        """flow-filter stage 1; priority = rule_priority(prefix, pf)
        (flow-filter/src/context/tables.rs:452-454)."""
        fam = ipaddress.ip_network(dst_prefix).version
        plen = ipaddress.ip_network(dst_prefix).prefixlen
        prio = ((plen + 1) << 1) | int(port_forwarding)
        self.ff_remote[fam].append(self.rule(fam, proto=proto, vni_a=src_vni, vni_b=gate_vni,
                                             dst=dst_prefix, dports=dports, priority=prio,
                                             action=dst_vni, action2=dst_nat))

    def add_ff_local(self, src_vni: int, dst_vni: int, src_prefix: str, src_nat: int = NAT_NONE,
                     proto: Optional[int] = None, sports=(0, 65535), gate: int = 0) -> None:
        fam = ipaddress.ip_network(src_prefix).version
        plen = ipaddress.ip_network(src_prefix).prefixlen
        self.ff_local[fam].append(self.rule(fam, proto=proto, vni_a=src_vni, vni_b=dst_vni,
                                            gate=gate, src=src_prefix, sports=sports,
                                            priority=(plen + 1) << 1, action=src_nat))

    # -- port forwarding -------------------------------------------------------
    def add_portfw(self, src_vni: int, proto: int, dst_vni: int, ext_prefix: str, int_prefix: str,
                   ext_ports, int_ports, init_timeout_s: int = 0, estab_timeout_s: int = 0) -> None:
        """PortFwEntry::new(PortFwKey(src_vpcd, proto), dst_vpcd, ext, int, ext_ports,
        int_ports, init, estab) (nat/src/portfw/portfwtable/objects.rs:70-103);
        proto 6 (TCP) or 17 (UDP), timeouts in seconds (0: the defaults)."""
        r = A.PortFwRule()
        r.src_vni, r.proto, r.dst_vni = src_vni, proto, dst_vni
        r.ext_lo, r.ext_hi = ext_ports
        r.int_lo, r.int_hi = int_ports
        r.init_timeout_s, r.estab_timeout_s = init_timeout_s, estab_timeout_s
        # Prefix::from_str keeps the host bits out (70.71.72.70/24 is 70.71.72.0/24)
        r.ext_prefix = mk_prefix(str(ipaddress.ip_network(ext_prefix, strict=False)))
        r.int_prefix = mk_prefix(str(ipaddress.ip_network(int_prefix, strict=False)))
        self.portfw.append(r)

    # -- masquerade -------------------------------------------------------------
    def add_masquerade(self, src_vni: int, dst_vni: int, private: Sequence[str],
                       public: Sequence[str], idle_timeout_s: int = 0,
                       claims: Sequence[Tuple[str, int, int, int]] = ()) -> None:
        """A masquerade expose of the peering src_vni -> dst_vni (VpcExpose::
        make_masquerade(idle).ip(private...).as_range(public...)); `claims`: the
        port-forwarding exposes of the same local manifest as (public prefix,
        lo, hi, protos) with protos of A.MASQ_TCP | A.MASQ_UDP."""
        e = A.MasqExpose(src_vni=src_vni, dst_vni=dst_vni, idle_timeout_s=idle_timeout_s)
        e.first_prefix = len(self.masq_prefixes)
        for p in private:
            self.masq_prefixes.append(mk_prefix(str(ipaddress.ip_network(p, strict=False))))
        for p in public:
            self.masq_prefixes.append(mk_prefix(str(ipaddress.ip_network(p, strict=False))))
        e.n_private, e.n_public = len(private), len(public)
        e.first_claim = len(self.masq_claims)
        for (pfx, lo, hi, protos) in claims:
            self.masq_claims.append(A.MasqClaim(prefix=mk_prefix(str(ipaddress.ip_network(pfx, strict=False))),
                                                lo=lo, hi=hi, protos=protos))
        e.n_claims = len(claims)
        self.masq.append(e)

    # -- static NAT -------------------------------------------------------------
    def add_nat_table(self, kind: int, src_vni: int, dst_vni: int,
                      entries: Sequence[dict]) -> None:
        """kind 0: dst_nat of PerVniTable(src_vni); kind 1: src_nat[dst_vni].
        Each entry: dict(prefix, pat=False, port_ranges=[(lo,hi)], size,
        ranges=[(orig_lo_ip, orig_lo_port, orig_hi_ip, orig_hi_port, tgt_lo_ip, tgt_hi_ip,
        tgt_lo_port, tgt_hi_port, offset)])."""
        first = len(self.nat_entries)
        for e in entries:
            ne = A.NatEntry()
            ne.prefix = mk_prefix(e["prefix"])
            ne.is_pat = 1 if e.get("pat") else 0
            ne.first_port_range = len(self.nat_prs)
            for lo, hi in e.get("port_ranges", []):
                self.nat_prs.append(A.PortRange(lo, hi))
            ne.n_port_ranges = len(self.nat_prs) - ne.first_port_range
            ne.first_range = len(self.nat_ranges)
            for (olo, olop, ohi, ohip, tlo, thi, tlop, thip, off) in e["ranges"]:
                r = A.NatRange()
                for k, x in enumerate(ip_obj(olo).packed):
                    r.orig_lo_ip[k] = x
                for k, x in enumerate(ip_obj(ohi).packed):
                    r.orig_hi_ip[k] = x
                for k, x in enumerate(ip_obj(tlo).packed):
                    r.tgt_lo_ip[k] = x
                for k, x in enumerate(ip_obj(thi).packed):
                    r.tgt_hi_ip[k] = x
                r.orig_lo_port, r.orig_hi_port = olop, ohip
                r.tgt_lo_port, r.tgt_hi_port = tlop, thip
                r.offset = off
                self.nat_ranges.append(r)
            ne.n_ranges = len(self.nat_ranges) - ne.first_range
            ne.size = e["size"]
            self.nat_entries.append(ne)
        self.nat_tables.append(A.NatTable(kind, src_vni, dst_vni, first,
                                          len(self.nat_entries) - first))

    # -- descriptor ----------------------------------------------------------
    def _arr(self, t, items):
        a = (t * max(1, len(items)))(*items)
        self._keep.append(a)
        return C.cast(a, C.POINTER(t)), len(items)

    def build(self):
        """Returns a POINTER(TablesDesc) valid while this builder lives."""
        d = A.TablesDesc()
        d.abi_version = A.ABI_VERSION
        d.genid = self.genid
        d.fibs, d.n_fibs = self._arr(A.Fib, self.fibs)
        d.vni_fibs, d.n_vni_fibs = self._arr(A.VniFib, self.vnis)
        d.routes, d.n_routes = self._arr(A.Route, self.routes)
        d.route_nhs, d.n_route_nhs = self._arr(A.RouteNh, self.nhs)
        d.entries, d.n_entries = self._arr(A.FibEntry, self.entries)
        d.instrs, d.n_instrs = self._arr(A.Instr, self.instrs)
        d.ifaces, d.n_ifaces = self._arr(A.Iface, self.ifaces)
        d.adjs, d.n_adjs = self._arr(A.Adjacency, self.adjs)
        d.acl_v4, d.n_acl_v4 = self._arr(A.Rule, self.acl[4])
        d.acl_v6, d.n_acl_v6 = self._arr(A.Rule, self.acl[6])
        d.acl_defaults, d.n_acl_defaults = self._arr(A.AclDefault, self.acl_defaults)
        d.ff_remote_v4, d.n_ff_remote_v4 = self._arr(A.Rule, self.ff_remote[4])
        d.ff_local_v4, d.n_ff_local_v4 = self._arr(A.Rule, self.ff_local[4])
        d.ff_remote_v6, d.n_ff_remote_v6 = self._arr(A.Rule, self.ff_remote[6])
        d.ff_local_v6, d.n_ff_local_v6 = self._arr(A.Rule, self.ff_local[6])
        d.nat_tables, d.n_nat_tables = self._arr(A.NatTable, self.nat_tables)
        d.nat_entries, d.n_nat_entries = self._arr(A.NatEntry, self.nat_entries)
        d.nat_port_ranges, d.n_nat_port_ranges = self._arr(A.PortRange, self.nat_prs)
        d.nat_ranges, d.n_nat_ranges = self._arr(A.NatRange, self.nat_ranges)
        d.portfw, d.n_portfw = self._arr(A.PortFwRule, self.portfw)
        d.masq, d.n_masq = self._arr(A.MasqExpose, self.masq)
        d.masq_prefixes, d.n_masq_prefixes = self._arr(A.Prefix, self.masq_prefixes)
        d.masq_claims, d.n_masq_claims = self._arr(A.MasqClaim, self.masq_claims)
        d.masq_config_tag = self.masq_config_tag
        d.masq_randomize = 1 if self.masq_randomize else 0
        d.masq_seed = self.masq_seed
        self._desc = d
        return C.pointer(d)
