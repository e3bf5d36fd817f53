"""Seeded port-forwarding bursts (test infrastructure): many connections
through a few port-forwarding rules, in bursts that mix what makes
PortForwarder order-dependent within a burst -- first packets (flow-pair
creation), repeats of a first packet (a second creation replaces the pair),
replies on the reverse flows, TCP handshakes and teardowns (NatFlowStatus),
resets, packets no rule covers, non-initial TCP segments without a flow,
and a rule-set change between bursts (stale-rule revalidation) -- so the
GPU's sequential port-forwarding pass can be compared bit for bit with the
oracle burst by burst."""
from __future__ import annotations

import ipaddress
import random
from typing import List, Tuple

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.flows import flow_key
from golden import pfkat
from golden.pfkat import ACK, FIN, PSH, RST, SYN, VPC1, VPC2, Pkt, frame

RULES = [
    # (proto, ext prefix, int prefix, ext ports, int ports)
    (6, "70.71.72.0/24", "192.168.1.0/24", (3000, 3099), (1000, 1099)),
    (6, "70.71.72.73/32", "192.168.9.9/32", (4000, 4000), (22, 22)),
    (17, "70.71.72.0/24", "192.168.2.0/24", (5000, 5199), (53, 252)),
    (17, "70.71.72.128/25", "192.168.3.0/25", (6000, 6009), (6000, 6009)),
]


def rules(which=None) -> List[dict]:
    out = []
    for k, (p, e, i, ep, ip) in enumerate(RULES):
        if which is not None and k not in which:
            continue
        out.append(dict(src_vni=VPC1, proto=p, dst_vni=VPC2, ext_prefix=e, int_prefix=i,
                        ext_ports=ep, int_ports=ip, init_timeout_s=10 + k, estab_timeout_s=100 + k))
    return out


def _map(rule, dst: str, dport: int) -> Tuple[str, int]:
    p, e, i, ep, ip = rule
    off = int(ipaddress.ip_address(dst)) - int(ipaddress.ip_network(e).network_address)
    return str(ipaddress.ip_address(int(ipaddress.ip_network(i).network_address) + off)), \
        ip[0] + dport - ep[0]


class Conn:
    def __init__(self, rng: random.Random, k: int):
        self.rule = RULES[rng.randrange(len(RULES))]
        p, e, i, ep, ip = self.rule
        net = ipaddress.ip_network(e)
        self.proto = p
        self.client = f"10.{(k >> 8) & 255}.{k & 255}.{1 + rng.randrange(200)}"
        self.cport = 1024 + rng.randrange(60000)
        self.dst = str(net.network_address + rng.randrange(net.num_addresses))
        self.dport = rng.randrange(ep[0], ep[1] + 1)
        self.srv, self.sport = _map(self.rule, self.dst, self.dport)

    def fwd(self, flags=0) -> Pkt:
        return Pkt(frame(self.client, self.dst, self.proto, self.cport, self.dport, flags), VPC1)

    def rev(self, flags=0) -> Pkt:
        return Pkt(frame(self.srv, self.client, self.proto, self.sport, self.cport, flags), VPC2)

    def keys(self):
        kind = A.FLOW_TCP if self.proto == 6 else A.FLOW_UDP
        return [flow_key(VPC1, self.client, self.dst, kind, self.cport, self.dport),
                flow_key(VPC2, self.srv, self.client, kind, self.sport, self.cport)]


def bursts(seed: int, n_conn: int = 400):
    """([(rules or None, [Pkt...])...], [flow keys]): three bursts on one
    rule set, a rule-set change, a fourth burst."""
    rng = random.Random(seed)
    cs = [Conn(rng, k) for k in range(n_conn)]
    b1, b2, b3, b4 = [], [], [], []
    for c in cs:
        t = c.proto == 6
        r = rng.random()
        if r < 0.05:                       # no rule covers it (a port outside every range)
            b1.append(Pkt(frame(c.client, c.dst, c.proto, c.cport, 2999 if t else 4999,
                                SYN if t else 0), VPC1))
            continue
        if t and r < 0.10:                 # not a first segment and no flow
            b1.append(c.fwd(ACK))
            continue
        b1.append(c.fwd(SYN if t else 0))
        if rng.random() < 0.1:             # the first packet twice in one burst
            b1.append(c.fwd(SYN if t else 0))
        # burst 2: the reply, then maybe the handshake's last ACK, data
        b2.append(c.rev(SYN | ACK if t else 0))
        if rng.random() < 0.7:
            b2.append(c.fwd(ACK if t else 0))
        if rng.random() < 0.3:
            b2.append(c.rev(ACK | PSH if t else 0))
        # burst 3: data, teardowns, resets
        x = rng.random()
        if t and x < 0.2:
            b3 += [c.fwd(FIN | ACK), c.rev(ACK), c.rev(FIN | ACK), c.fwd(ACK)]
        elif t and x < 0.3:
            b3 += [c.rev(FIN | ACK), c.fwd(FIN | ACK), c.rev(ACK)]
        elif t and x < 0.4:
            b3 += [c.fwd(RST), c.fwd(ACK)]
        else:
            b3 += [c.fwd(ACK if t else 0), c.rev(ACK if t else 0)]
        b4 += [c.fwd(ACK if t else 0), c.rev(ACK if t else 0)]
    for b in (b1, b2, b3, b4):
        rng.shuffle(b)
    keys = [k for c in cs for k in c.keys()]
    return [(None, b1), (None, b2), (None, b3), (rules([0, 2, 3]), b4)], keys


def run(r, seed: int, n_conn: int, capacity=None, on_burst=None):
    """All bursts of `bursts(seed)` on runner r (pfkat.OracleRunner /
    GpuRunner); on_burst(k, res, buf, infos, lookups) after each."""
    plan, keys = bursts(seed, n_conn)
    r.publish(pfkat.world(rules())())
    if capacity is not None:
        (r.fl if hasattr(r, "fl") else r.ft).set_capacity(capacity)
    now = 0
    from edgecase import pack_burst
    for k, (rs, pk) in enumerate(plan):
        now += 5 * pfkat.SEC
        r.set_clock(now)
        if rs is not None:
            r.publish(pfkat.world(rs)())
        buf, inp = pack_burst([(p.frame, 1, A.IN_SEEDED_OVERLAY, p.vni) for p in pk])
        res = r.burst(buf, inp)
        refs = res["flow_ref"]
        infos = r.get(refs)
        keyarr = np.array(keys, dtype=A.FLOW_KEY)
        look = (r.fl if hasattr(r, "fl") else r.ft).lookup(keyarr)
        if on_burst:
            on_burst(k, res, buf, infos, look)
