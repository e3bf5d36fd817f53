"""Shared test helpers: compare two runs of the path (GPU / emulation vs oracle)."""
import numpy as np

from dataplane_amd import _abi as A


def compare(out_ref, buf_ref, out_dut, buf_dut, inp, label=""):
    """Bit-exact: every dp_pkt_out_t field (and every dp_pkt_meta_t field when
    both sides carry one -- PKT_RES records), and every serialized byte of
    every Delivered packet (plus the whole buffer, which also pins that
    nothing else was touched)."""
    out_ref, out_dut = common_fields(out_ref, out_dut)
    mism = np.nonzero(out_ref != out_dut)[0]
    msg = []
    for i in mism[:5]:
        msg.append(f"pkt {i}: ref {out_ref[i]} dut {out_dut[i]}")
    assert len(mism) == 0, f"{label}: {len(mism)} metadata mismatches\n" + "\n".join(msg)
    deliv = np.nonzero(out_ref["done"] == A.DONE["Delivered"])[0]
    for i in deliv:
        o, l = int(out_ref[i]["off"]), int(out_ref[i]["len"])
        if not np.array_equal(buf_ref[o:o + l], buf_dut[o:o + l]):
            d = np.nonzero(buf_ref[o:o + l] != buf_dut[o:o + l])[0]
            raise AssertionError(f"{label}: pkt {i} bytes differ at {d[:8]}")
    # A dropped packet's buffer is released by the reference (its bytes are
    # unobservable; e.g. Packet::vxlan_encap has already prepended the inner
    # headers when Egress then fails), so its slot is excluded.  Everything
    # else -- delivered frames, their headroom, gaps -- must match.
    # A packet owns [off - DP_HEADROOM, off + len) whatever the buffer layout
    # (packed: 96 B headroom; DPDK mbuf: 128 B in front of the frame).
    diff = buf_ref != buf_dut
    dropped = np.nonzero(out_ref["done"] != A.DONE["Delivered"])[0]
    if len(dropped):
        starts = inp["off"].astype(np.int64) - A.HEADROOM
        ends = inp["off"].astype(np.int64) + inp["len"].astype(np.int64)
        for i in dropped:
            diff[starts[i]:ends[i]] = False
    if diff.any():
        d = np.nonzero(diff)[0]
        owner = int(np.searchsorted(inp["off"].astype(np.int64) - A.HEADROOM, d[0], "right")) - 1
        raise AssertionError(f"{label}: buffers differ outside delivered frames at {d[:8]} "
                             f"(packet {owner}: {out_ref[owner]} / {out_dut[owner]})")


def compare_bulk(out_ref, buf_ref, out_dut, buf_dut, inp, label=""):
    """compare() for large bursts, vectorised: every dp_pkt_out_t field, and
    the whole buffer outside the slots of dropped packets (which holds every
    byte of every delivered frame)."""
    a, b = common_fields(out_ref, out_dut)
    mism = np.nonzero(a != b)[0]
    assert len(mism) == 0, f"{label}: {len(mism)} records differ, first pkt {mism[0]}: {a[mism[0]]} vs {b[mism[0]]}"
    diff = buf_ref != buf_dut
    dropped = np.nonzero(out_ref["done"] != A.DONE["Delivered"])[0]
    if len(dropped):
        mark = np.zeros(len(diff) + 1, np.int32)
        s = (inp["off"][dropped].astype(np.int64) - A.HEADROOM).clip(0)
        e = inp["off"][dropped].astype(np.int64) + inp["len"][dropped].astype(np.int64)
        np.add.at(mark, s, 1)
        np.add.at(mark, e, -1)
        diff &= np.cumsum(mark)[:-1] == 0
    if diff.any():
        d = np.nonzero(diff)[0]
        owner = int(np.searchsorted(inp["off"].astype(np.int64) - A.HEADROOM, d[0], "right")) - 1
        raise AssertionError(f"{label}: buffers differ at {d[:8]} (packet {owner}: {out_ref[owner]} / {out_dut[owner]})")


def common_fields(a, b):
    """Both record arrays projected onto the fields they share (a device run
    without a meta array yields dp_pkt_out_t alone).  flow_ref is left out:
    the oracle's refs and the device table's are different handle spaces,
    which the flow tests match up through the flows they name."""
    names = [n for n in a.dtype.names if n in b.dtype.names and n not in ("pad", "flow_ref")]
    return a[names], b[names]


def field_diff(a, b, k):
    """Indices of records whose field k differs (array fields such as nh_addr
    compare whole rows)."""
    d = a[k] != b[k]
    if d.ndim > 1:
        d = d.reshape(len(d), -1).any(axis=1)
    return d


def hist(out):
    h = np.bincount(out["done"].astype(np.int64), minlength=256)
    return {A.DONE_NAMES[i] if i < A.DONE_COUNT else str(i): int(c) for i, c in enumerate(h) if c}
