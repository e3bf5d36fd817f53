"""The flow-filter classifier alone (dp_ff_classify, SURVEY.md §8b: the
narrower drop-in for A13 -- FlowFilterContext::lookup_batch, flow-filter/src/
context/tables.rs:800-848, and the two rte_acl tables behind it).

CPU: the reference's own context KATs (flow-filter/src/context/tests.rs, as
tests/golden/ffkat.py) through the oracle's classify (dpo_ff_classify); the
oracle's classify is the stage (the flow filter the oracle's whole path runs
gave the same packets the same verdicts); the conversion of the reference's
key bytes (dp_ff_key_from_match: RemoteKey / LocalKey::as_key, host code)
pinned against a restatement of MatchKey::as_key_into's layout.
GPU (tests/test_gpu_ff_classify.py): the same through the C ABI."""
import ctypes as C
import struct

import numpy as np
import pytest

from dataplane_amd import _abi as A
from golden import ffkat
from oracle.pyoracle import Oracle


@pytest.mark.parametrize("case", ffkat.cases(), ids=lambda c: c.name)
def test_oracle_ff_kat(case):
    t = ffkat.tables(case)
    o = Oracle(t.build())
    try:
        res = o.ff_classify(ffkat.inputs(case.probes))
    finally:
        o.close()
    errs = ffkat.check(case, res)
    assert not errs, "\n".join(errs)


def remote_key(q) -> bytes:
    """RemoteKey::as_key (tables.rs:192-207 through match-action-derive/src/
    lib.rs:191-206): proto (1 B), src_vni and dst_vni (GateVni; Vni as 4 B,
    net/src/fixed_size.rs:61-74), destination, destination port, big-endian,
    back to back."""
    al = 4 if int(q["dst_family"]) == 4 else 16
    return (struct.pack(">BII", int(q["proto"]), int(q["src_vni"]), int(q["dst_vni"])) + bytes(q["dst"][:al]) +
            struct.pack(">H", int(q["dport"])))


def local_key(q) -> bytes:
    """LocalKey::as_key (tables.rs:211-229): proto, src_vni, dst_vni, source,
    source port, gate (SourceGate, 1 B: tables.rs:171-180)."""
    al = 4 if int(q["src_family"]) == 4 else 16
    return (struct.pack(">BII", int(q["proto"]), int(q["src_vni"]), int(q["dst_vni"])) + bytes(q["src"][:al]) +
            struct.pack(">HB", int(q["sport"]), int(q["gate"])))


def random_inputs(n: int, seed: int) -> np.ndarray:
    r = np.random.default_rng(seed)
    q = np.zeros(n, A.FF_INPUT)
    fam = np.where(r.random(n) < 0.5, 4, 6)
    q["src_family"] = q["dst_family"] = fam
    q["proto"] = r.choice([1, 6, 17, 58], n)
    q["gate"] = r.integers(0, 2, n)
    q["src_vni"] = r.integers(1, 1 << 24, n)
    q["dst_vni"] = r.integers(0, 1 << 24, n)
    q["sport"] = r.integers(0, 65536, n)
    q["dport"] = r.integers(0, 65536, n)
    q["src"] = r.integers(0, 256, (n, 16))
    q["dst"] = r.integers(0, 256, (n, 16))
    q["src"][fam == 4, 4:] = 0
    q["dst"][fam == 4, 4:] = 0
    return q


def match_buf(keys: list, stride: int) -> np.ndarray:
    size = len(keys[0])
    buf = np.zeros(len(keys) * stride, np.uint8)
    for i, k in enumerate(keys):
        buf[i * stride:i * stride + size] = np.frombuffer(k, np.uint8)
    return buf


@pytest.mark.parametrize("stride", [0, 32])
def test_ff_key_from_match(stride):
    lib = A.gpu_lib()  # (host code of the library: no device is touched)
    q = random_inputs(400, 11 + stride)
    for table, mk in ((A.FF_REMOTE, remote_key), (A.FF_LOCAL, local_key)):
        for fam in (4, 6):
            sel = q[q["src_family"] == fam]
            keys = [mk(k) for k in sel]
            size = len(keys[0])
            want_size = {(A.FF_REMOTE, 4): A.FF_REMOTE_KEY_V4, (A.FF_REMOTE, 6): A.FF_REMOTE_KEY_V6,
                         (A.FF_LOCAL, 4): A.FF_LOCAL_KEY_V4, (A.FF_LOCAL, 6): A.FF_LOCAL_KEY_V6}[(table, fam)]
            assert size == want_size
            st = stride or size
            buf = match_buf(keys, st)
            got = np.zeros(len(sel), A.FF_INPUT)
            assert lib.dp_ff_key_from_match(table, buf.ctypes.data, size, st, len(sel), got.ctypes.data) == 0
            exp = sel.copy()
            # a remote key carries no source (nor source port / gate), a local
            # key no destination (nor destination port)
            if table == A.FF_REMOTE:
                exp["src"], exp["sport"], exp["gate"] = 0, 0, 0
            else:
                exp["dst"], exp["dport"] = 0, 0
            assert got.tobytes() == exp.tobytes()
    out = np.zeros(1, A.FF_INPUT)
    buf = np.zeros(64, np.uint8)
    assert lib.dp_ff_key_from_match(A.FF_REMOTE, buf.ctypes.data, 16, 16, 1, out.ctypes.data) == -22
    assert lib.dp_ff_key_from_match(A.FF_LOCAL, buf.ctypes.data, 15, 15, 1, out.ctypes.data) == -22
    assert lib.dp_ff_key_from_match(A.FF_LOCAL, buf.ctypes.data, 16, 15, 1, out.ctypes.data) == -22
    assert lib.dp_ff_key_from_match(3, buf.ctypes.data, 15, 15, 1, out.ctypes.data) == -22
    assert lib.dp_ff_key_from_match(A.FF_REMOTE, C.c_void_p(0), 27, 27, 0, C.c_void_p(0)) == 0


def ff_inputs_of(w, res):
    """The LookupInput of every overlay packet the flow filter consulted (the
    oracle's whole path: its out record names the verdict), as the stage asks
    it: ungated, the 5-tuple as received."""
    from test_acl_classify import keys_of
    idx, keys = keys_of(w, res, res)
    q = np.zeros(len(keys), A.FF_INPUT)
    q["src_vni"] = keys["src_vni"]
    q["src_family"] = q["dst_family"] = keys["family"]
    for f in ("proto", "sport", "dport", "src", "dst"):
        q[f] = keys[f]
    return idx, q


@pytest.mark.parametrize("cfg", [2, 5])
def test_oracle_ff_classify_is_the_stage(cfg):
    """Packets the whole path let through the flow filter: Route to the VPC
    their metadata names; stage 1 / stage 2 alone agree with the pair."""
    from dataplane_amd.workload import Workload
    w = Workload(cfg, 4000, seed=50 + cfg, n_routes_v4=2000, n_routes_v6=1000, n_acl=300, n_nat=16)
    o = Oracle(w.tables)
    res = o.process(w.fresh_buf(), w.inp)
    idx, q = ff_inputs_of(w, res)
    assert len(idx) > 1000
    got = o.ff_classify(q)
    assert (got["outcome"] == A.FF_ROUTE).all()
    assert np.array_equal(got["dst_vni"], res["dst_vni"][idx])
    r1 = o.ff_classify(q, stage=1)
    assert np.array_equal(r1["dst_vni"], got["dst_vni"]) and np.array_equal(r1["dst_nat"], got["dst_nat"])
    q2 = q.copy()
    q2["dst_vni"] = got["dst_vni"]
    r2 = o.ff_classify(q2, stage=2)
    assert (r2["outcome"] == A.FF_ROUTE).all() and np.array_equal(r2["src_nat"], got["src_nat"])
    o.close()
