"""Which input form a pipeline user must give the GPU block.

The reference runs its stages on `Packet::new(raw frame)` and serializes at
transmit.  The C ABI takes the raw frame.  A `NetworkFunction` adapter
placed inside a `DynPipeline` would receive `Packet`s instead and would have
to hand the GPU `Packet::serialize(Packet::new(raw))` -- a different frame
wherever serialize normalizes what it re-emits.  This test runs the edge
corpus both ways through the oracle (and the second form through the
kernel's host build too) and pins exactly which packets come out different:

- ICMP error messages whose ICMP / embedded IPv4 checksum is wrong: the
  IcmpErrorHandler drops them InvalidChecksum (nat/src/icmp_handler/nf.rs:
  61-120); serialize recomputes the checksums first, so they go on;
- frames beyond the parse limits (a fifth VLAN tag, a fourth IPv6 extension
  header, net/src/headers/mod.rs:492-500): consumed, not kept, so not
  re-emitted;
- fields the path carries through untouched when nothing asks for a
  checksum refresh (checksums, reserved bits of the corpus's mutated
  frames): serialize rewrites them on the way in.

Every difference is confined to frames that serialize changes, and the
raw-frame form is the one equal to the reference; hence the hook before
Packet::new."""
from collections import Counter

import numpy as np

from dataplane_amd import _abi as A
from edgecase import edge_frames, edge_tables, pack_burst
from helpers import compare
from oracle.pyoracle import Oracle, reserialize
import pyemu


def _vlans(f: bytes) -> int:
    n, o = 0, 12
    while f[o:o + 2] in (b"\x81\x00", b"\x88\xa8"):
        n, o = n + 1, o + 4
    return n


def test_raw_vs_serialized_packet_input():
    tp = edge_tables().build()
    frames = edge_frames(12000, 7)
    again = [reserialize(f[0]) for f in frames]
    keep = [i for i, a in enumerate(again) if a is not None]  # Packet::new succeeds
    raw = [frames[i] for i in keep]
    ser = [(again[i],) + tuple(frames[i][1:]) for i in keep]
    changed = np.array([again[i] != frames[i][0] for i in keep])
    ba, ia = pack_burst(raw)
    bs, is_ = pack_burst(ser)
    oa = Oracle(tp).process(ba, ia)
    bs_emu = bs.copy()
    os_ = Oracle(tp).process(bs, is_)
    # the kernel body on the serialized form equals the oracle there too
    compare(os_, bs, pyemu.process(tp, bs_emu, is_), bs_emu, is_, "serialized input form")

    def frame(o, b):
        return bytes(b[o["off"]:o["off"] + o["len"]]) if o["done"] == A.DONE["Delivered"] else b""

    diff = [k for k in range(len(keep))
            if oa[k]["done"] != os_[k]["done"] or oa[k]["meta_flags"] != os_[k]["meta_flags"]
            or frame(oa[k], ba) != frame(os_[k], bs)]
    assert diff, "the corpus should contain frames serialize normalizes"
    classes = Counter()
    for k in diff:
        assert changed[k], f"packet {k}: same input frame, different outcome"
        f, g = raw[k][0], ser[k][0]
        if oa[k]["done"] == A.DONE["InvalidChecksum"]:
            classes["icmp error, bad checksum"] += 1
        elif len(f) != len(g) and (_vlans(f) > 4 or f[12:14] == b"\x86\xdd" or _vlans(f) and
                                   f[12 + 4 * _vlans(f):14 + 4 * _vlans(f)] == b"\x86\xdd"):
            classes["headers past the parse limits"] += 1
        else:
            assert oa[k]["done"] == os_[k]["done"] == A.DONE["Delivered"], (k, oa[k], os_[k])
            assert len(f) == len(g), k
            classes["field normalized by serialize"] += 1
    assert classes["icmp error, bad checksum"] > 0
    # a small share of the corpus (which is built from edge cases)
    assert len(diff) < 0.02 * len(keep), classes
    print(dict(classes), "of", len(keep))
