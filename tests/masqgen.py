"""Seeded masquerade bursts (test infrastructure): many connections from two
VPCs masqueraded towards a third, in bursts that mix what makes Masquerade
order-dependent within a burst -- first packets (allocations from a shared,
port-forwarding-claimed public range small enough to run out), repeats of a
first packet (the second pair replaces the first; its allocation goes back
when the burst ends), replies on the reverse flows, TCP handshakes,
teardowns and resets, DNS answers (a UDP reply from port 53 closes the
flow), ICMP echo (identifiers), packets no expose covers, non-initial TCP
segments without a flow -- and, between bursts, timer sweeps (expired flows
give their ports back), a republish of the same config (generation upgrade),
a narrowed config (the allocator is rebuilt and the flows it still serves
re-reserved; the others invalidated) and no masquerade at all.  The GPU's
sequential NAT pass is compared with the oracle bit for bit, burst by burst
(tests/test_gpu_masquerade.py)."""
from __future__ import annotations

import random
from typing import List

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.flows import flow_key
from edgecase import pack_burst
from golden import masqkat as M
from golden.masqkat import ACK, FIN, PSH, RST, SYN, SEC, V1, V2, V3, Pkt

# two exposes share 2.2.2.0/31 (regions by sharers); port-forwarding claims
# leave each address 535 TCP ports and 76 UDP ports
CLAIMS = [("2.2.2.0/31", 1024, 65000, A.MASQ_TCP), ("2.2.2.0/31", 1100, 65535, A.MASQ_UDP)]
M.OVERLAYS.setdefault("gen", lambda: [
    (V1, V2, ["1.1.0.0/16"], ["2.2.2.0/31"], 30),
    (V3, V2, ["1.3.0.0/16"], ["2.2.2.0/31", "2.2.3.0/30"], 0),
])
M.OVERLAYS.setdefault("gen_narrow", lambda: [
    (V3, V2, ["1.3.0.0/16"], ["2.2.2.0/31", "2.2.3.0/30"], 0),
])
PEERS = [(V1, V2), (V3, V2), (V2, V1), (V2, V3)]


def world(overlay: str, genid: int, randomize_seed=None):
    t = M.world(overlay, genid, PEERS)
    if randomize_seed is not None:  # MasqueradeConfig::set_randomize(true)
        t.masq_randomize, t.masq_seed = True, randomize_seed
    # the claims ride on the exposes of 2.2.2.0/31 (rebuild them with claims)
    t.masq, t.masq_prefixes, t.masq_claims = [], [], []
    for (s, d, priv, pub, idle) in M.OVERLAYS[overlay]():
        cl = [(p, lo, hi, pr) for (p, lo, hi, pr) in CLAIMS if p in pub]
        t.add_masquerade(s, d, priv, pub, idle_timeout_s=idle, claims=cl)
    return t


class Conn:
    def __init__(self, rng: random.Random, k: int):
        self.vni = V1 if rng.random() < 0.6 else V3
        net = "1.1" if self.vni == V1 else "1.3"
        if rng.random() < 0.04:
            net = "1.9"  # no expose covers it: Denied
        self.src = f"{net}.{(k >> 8) & 255}.{k & 255}"
        r = rng.random()
        self.proto = 6 if r < 0.55 else 17 if r < 0.85 else 1
        self.sport = 1024 + rng.randrange(60000)
        self.dst = f"5.0.{rng.randrange(4)}.{1 + rng.randrange(200)}"
        self.dport = 53 if (self.proto == 17 and rng.random() < 0.2) else 80 + rng.randrange(4)
        self.ident = rng.randrange(65536)

    def fwd(self, flags=0) -> Pkt:
        if self.proto == 1:
            return Pkt(M.echo_frame(self.src, self.dst, self.ident), self.vni)
        return Pkt(M.l4_frame(self.src, self.dst, self.proto, self.sport, self.dport, flags), self.vni)

    def key(self):
        kind = {6: A.FLOW_TCP, 17: A.FLOW_UDP, 1: A.FLOW_ICMP_QUERY}[self.proto]
        if self.proto == 1:
            return flow_key(self.vni, self.src, self.dst, kind, self.ident, 0)
        return flow_key(self.vni, self.src, self.dst, kind, self.sport, self.dport)


def rev_of(c: Conn, out: dict, flags=0) -> Pkt:
    """The peer's answer to the translated packet `out` (its fields)."""
    if c.proto == 1:
        return Pkt(M.echo_frame(out["dst"], out["src"], out["ident"], reply=True), V2)
    return Pkt(M.l4_frame(out["dst"], out["src"], c.proto, out["dport"], out["sport"], flags), V2)


def run(r, seed: int, n_conn: int, capacity=None, on_burst=None, before_burst=None, randomize_seed=None):
    """The bursts of one seed on runner r (masqkat.OracleRunner / GpuRunner);
    on_burst(k, res, buf, infos, lookups, related_infos) after each.  Replies
    are built from the runner's own translated packets.  randomize_seed: the
    allocator shuffles each address's port blocks (dpgpu.h masq_randomize)."""
    rng = random.Random(seed)
    cs = [Conn(rng, k) for k in range(n_conn)]
    r.publish(world("gen", 1, randomize_seed))
    if capacity is not None:
        (r.fl if hasattr(r, "fl") else r.ft).set_capacity(capacity)
    keys = np.array([c.key() for c in cs], dtype=A.FLOW_KEY)
    outs = {}  # connection -> its last translated forward packet
    now = 0
    # (clock advance, publish, sweep, packet plan)
    def first(c):
        t = c.proto == 6
        if t and rng.random() < 0.05:
            return [(c, "fwd", ACK)]  # not a first segment, no flow
        pk = [(c, "fwd", SYN if t else 0)]
        if rng.random() < 0.1:
            pk.append((c, "fwd", SYN if t else 0))  # the first packet twice
        return pk

    def answer(c):
        t = c.proto == 6
        pk = [(c, "rev", SYN | ACK if t else 0)]
        if rng.random() < 0.7:
            pk.append((c, "fwd", ACK if t else 0))
        if rng.random() < 0.3:
            pk.append((c, "rev", ACK | PSH if t else 0))
        return pk

    def later(c):
        t = c.proto == 6
        x = rng.random()
        if t and x < 0.2:
            return [(c, "fwd", FIN | ACK), (c, "rev", ACK), (c, "rev", FIN | ACK), (c, "fwd", ACK)]
        if t and x < 0.3:
            return [(c, "rev", FIN | ACK), (c, "fwd", FIN | ACK), (c, "rev", ACK)]
        if t and x < 0.4:
            return [(c, "fwd", RST), (c, "fwd", ACK)]
        return [(c, "fwd", ACK if t else 0), (c, "rev", ACK if t else 0)]

    half = cs[: n_conn // 2]
    rest = cs[n_conn // 2:]
    plan = [
        (SEC, None, False, [p for c in half for p in first(c)]),
        (SEC, None, False, [p for c in half for p in answer(c)]),
        (SEC, None, False, [p for c in half for p in later(c)] + [p for c in rest for p in first(c)]),
        # one-way flows (5 s) and closed ones leave; their tuples go back
        (6 * SEC, None, True, [p for c in rest for p in answer(c)] + [p for c in half for p in first(c)]),
        (SEC, ("gen", 2), False, [p for c in cs for p in later(c)]),
        (SEC, ("gen_narrow", 3), False, [p for c in cs for p in later(c)] + [p for c in half for p in first(c)]),
        (SEC, ("none", 4), True, [p for c in cs for p in later(c)]),
    ]
    for k, (adv, pub, sweep, pk) in enumerate(plan):
        now += adv
        r.set_clock(now)
        if pub is not None:
            r.publish(world(*pub, randomize_seed))
        if sweep:
            r.sweep(now)
        if before_burst:
            before_burst(k, r.lookup(keys))
        rng.shuffle(pk)
        pkts, who = [], []
        for (c, d, fl) in pk:
            if d == "rev":
                if id(c) not in outs:
                    continue
                pkts.append(rev_of(c, outs[id(c)], fl))
            else:
                pkts.append(c.fwd(fl))
            who.append((c, d))
        buf, inp = pack_burst([(p.frame, 1, A.IN_SEEDED_OVERLAY, p.vni) for p in pkts])
        res = r.burst(buf, inp)
        for i, (c, d) in enumerate(who):
            o = res[i]
            if d == "fwd" and o["done"] == A.DONE["Delivered"]:
                outs[id(c)] = M.out_fields(buf[o["off"]:o["off"] + o["len"]].tobytes())
        infos = r.get(res["flow_ref"])
        look = r.lookup(keys)
        rel = r.get(look["related"])
        if on_burst:
            on_burst(k, res, buf, infos, look, rel, pkts)
