"""Seeded flow-table scenarios over a synthetic workload (test infrastructure).

From a workload burst: pick packets, make flow pairs for their keys (the
request flow from the packet's VPC, the reply flow from its destination VPC)
with a mix of statuses, generations, destinations and NAT flags; build a
burst of those packets, their replies and repeats in a shuffled order, so one
burst exercises FlowLookup, the flow-filter bypass / invalidation, the ACL
reply path and the in-burst invalidation order together.
"""
from __future__ import annotations

import struct
from typing import List, Tuple

import numpy as np

from dataplane_amd import _abi as A
from dataplane_amd.flows import flow_key, make_flow, reverse_key
import ipaddress


def frame_key(frame: bytes, vni: int):
    """FlowKey of an untagged Eth / IPv4|IPv6 / TCP|UDP frame from VPC `vni`."""
    et = struct.unpack("!H", frame[12:14])[0]
    if et == 0x0800:
        ihl = (frame[14] & 0xF) * 4
        proto, src, dst, l4 = frame[23], frame[26:30], frame[30:34], 14 + ihl
    elif et == 0x86DD:
        proto, src, dst, l4 = frame[20], frame[22:38], frame[38:54], 54
    else:
        return None
    if proto not in (6, 17):
        return None
    sp, dp = struct.unpack("!HH", frame[l4:l4 + 4])
    if not sp or not dp:
        return None
    return flow_key(vni, ipaddress.ip_address(src), ipaddress.ip_address(dst),
                    A.FLOW_TCP if proto == 6 else A.FLOW_UDP, sp, dp)


def reply_frame(frame: bytes) -> bytes:
    """The same frame with addresses and ports swapped (its checksums stay
    valid: the one's-complement sums are order-independent)."""
    b = bytearray(frame)
    et = struct.unpack("!H", frame[12:14])[0]
    if et == 0x0800:
        ihl = (frame[14] & 0xF) * 4
        b[26:30], b[30:34] = frame[30:34], frame[26:30]
        l4 = 14 + ihl
    else:
        b[22:38], b[38:54] = frame[38:54], frame[22:38]
        l4 = 54
    b[l4:l4 + 2], b[l4 + 2:l4 + 4] = frame[l4 + 2:l4 + 4], frame[l4:l4 + 2]
    return bytes(b)


def frames_of(w) -> List[Tuple[bytes, int]]:
    return [(bytes(w.buf[int(r["off"]):int(r["off"]) + int(r["len"])]), int(r["src_vni"]))
            for r in w.inp]


def scenario(frames, dst_vnis, genid: int, seed: int, n_flows: int, vnis):
    """Flows to insert (as ('pair', a, b) / ('one', f) items, with the
    statuses to set after insertion) and the burst ((frame, vni) list)."""
    rng = np.random.default_rng(seed)
    cand = [i for i, (f, v) in enumerate(frames) if v and dst_vnis[i] and frame_key(f, v) is not None]
    rng.shuffle(cand)
    picked, seen = [], set()
    for i in cand:
        k = frame_key(*frames[i])
        kb = k.tobytes()
        rk = reverse_key(k, int(dst_vnis[i])).tobytes()
        if kb in seen or rk in seen:
            continue
        seen.update((kb, rk))
        picked.append(i)
        if len(picked) == n_flows:
            break

    def gen():
        return int(rng.choice([genid - 1, genid, genid, genid, genid + 1]))

    items, burst = [], []
    for i in picked:
        f, v = frames[i]
        d = int(dst_vnis[i])
        k = frame_key(f, v)
        dst_a = d if rng.random() < 0.85 else int(rng.choice(vnis))
        flags = int(rng.integers(0, 4)) << 1
        a = make_flow(k, dst_a, A.FLOW_INITIATOR | flags, gen())
        b = make_flow(reverse_key(k, d), v, flags, gen())
        st = [A.FLOW_ACTIVE, A.FLOW_ACTIVE]
        for j in range(2):
            if rng.random() < 0.15:
                st[j] = int(rng.choice([A.FLOW_CANCELLED, A.FLOW_DETACHED, A.FLOW_EXPIRED]))
        if rng.random() < 0.85:
            items.append(("pair", a, b, st))
        else:
            items.append(("one", a, st[:1]))
        # the request (sometimes twice) and the reply (sometimes twice)
        for _ in range(int(rng.integers(0, 3))):
            burst.append((f, v))
        for _ in range(int(rng.integers(0, 3))):
            burst.append((reply_frame(f), d))
    # packets with no flow
    for i in rng.choice(len(frames), size=min(len(frames), max(16, n_flows)), replace=False):
        burst.append(frames[int(i)])
    order = rng.permutation(len(burst))
    return items, [burst[int(j)] for j in order]


def install(ft, items):
    """Insert the scenario's flows into `ft`; returns the refs in insertion
    order (DP_FLOW_NONE for a refused flow)."""
    refs = []
    for it in items:
        if it[0] == "pair":
            r, _ = ft.insert_pair(it[1], it[2])
            sts = it[3]
        else:
            r, _ = ft.insert(it[1])
            sts = it[2]
        for ref, st in zip(r, sts):
            if int(ref) != A.FLOW_NONE and st != A.FLOW_ACTIVE:
                ft.set_status(int(ref), st)
        refs += [int(x) for x in r]
    return refs
