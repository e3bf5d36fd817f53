"""The ACL classifier alone (dp_acl_classify, SURVEY.md §8b: the batch
Lookup<K, A> of acl/src/dpdk/lookup.rs:112-155).

CPU: the oracle's classify (dpo_acl_classify) gives the ACL verdict and rule
the oracle's whole path gave the same packets (out.acl, acl_rule), over the
C2 and C5 workload shapes -- the checker is the stage.
GPU: dp_acl_classify through the C ABI == the oracle on those keys and on
perturbed ones (other ports, addresses, peerings: misses, defaults, peerings
without an ACL), both classifier forms, v4 and v6; and over the reference's own
key bytes (AclKey::as_key, dp_acl_classify_match) with BASELINE's 10k rules.
The conversion of those bytes (dp_acl_key_from_match, host code) is pinned on
the CPU against a restatement of MatchKey::as_key_into's layout."""
import struct

import numpy as np
import pytest

from dataplane_amd import _abi as A
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle


def keys_of(w: Workload, out, meta) -> np.ndarray:
    """The ACL key of every packet whose ACL was consulted (out.acl 1-5):
    the peering from its metadata, the 5-tuple from the frame as received
    (the ACL runs before static NAT; overlay frames, no VLAN / extension
    headers)."""
    ks = []
    for i in np.nonzero((out["acl"] >= 1) & (out["acl"] <= 5))[0]:
        o, ln = int(w.inp[i]["off"]), int(w.inp[i]["len"])
        fr = w.buf[o:o + ln]
        et = int(fr[12]) << 8 | int(fr[13])
        k = np.zeros((), A.ACL_KEY)
        k["src_vni"], k["dst_vni"] = meta[i]["src_vni"], meta[i]["dst_vni"]
        if et == 0x0800:
            ihl = (int(fr[14]) & 15) * 4
            k["family"], k["proto"] = 4, fr[23]
            k["src"][:4], k["dst"][:4] = fr[26:30], fr[30:34]
            l4 = 14 + ihl
        elif et == 0x86DD:
            k["family"], k["proto"] = 6, fr[20]
            k["src"][:], k["dst"][:] = fr[22:38], fr[38:54]
            l4 = 54
        else:
            continue
        if int(k["proto"]) in (6, 17):
            k["sport"] = int(fr[l4]) << 8 | int(fr[l4 + 1])
            k["dport"] = int(fr[l4 + 2]) << 8 | int(fr[l4 + 3])
        ks.append((i, k))
    idx = np.array([i for i, _ in ks])
    arr = np.array([k for _, k in ks], dtype=A.ACL_KEY)
    return idx, arr


def perturb(keys: np.ndarray, seed: int) -> np.ndarray:
    r = np.random.default_rng(seed)
    k = keys.copy()
    n = len(k)
    k["sport"] = np.where(r.random(n) < 0.5, r.integers(0, 65536, n), k["sport"])
    k["dport"] = np.where(r.random(n) < 0.5, r.integers(0, 65536, n), k["dport"])
    flip = r.random(n) < 0.3
    k["dst"][flip, 3] ^= r.integers(1, 256, int(flip.sum())).astype(np.uint8)
    swap = r.random(n) < 0.1
    k["src_vni"][swap], k["dst_vni"][swap] = k["dst_vni"][swap], k["src_vni"][swap].copy()
    odd = r.random(n) < 0.02
    k["family"][odd] = 5  # not classified
    return k


@pytest.mark.parametrize("cfg", [2, 5])
def test_oracle_classify_is_the_stage(cfg):
    w = Workload(cfg, 4000, seed=70 + cfg, n_routes_v4=2000, n_routes_v6=1000, n_acl=300, n_nat=16)
    o = Oracle(w.tables)
    b = w.fresh_buf()
    res = o.process(b, w.inp)
    idx, keys = keys_of(w, res, res)
    assert len(idx) > 1000
    got = o.acl_classify(keys)
    assert np.array_equal(got["acl"], res["acl"][idx])
    ruled = got["acl"] <= 2
    assert np.array_equal(got["rule"][ruled], res["acl_rule"][idx][ruled])
    assert set(np.unique(got["acl"]).tolist()) >= {1, 2}


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 5])
@pytest.mark.parametrize("form", ["list", "bv"])
def test_gpu_acl_classify(cfg, form, cls_form):
    from dataplane_amd import GpuPathNf
    w = Workload(cfg, 20000, seed=80 + cfg, n_routes_v4=4000, n_routes_v6=2000, n_acl=600, n_nat=16)
    o = Oracle(w.tables)
    res = o.process(w.fresh_buf(), w.inp)
    _, keys = keys_of(w, res, res)
    keys = np.concatenate([keys, perturb(keys, cfg)])
    want = o.acl_classify(keys)
    cls_form(A.gpu_lib(), form)
    nf = GpuPathNf(0)
    try:
        nf.publish(w.tables)
        got = nf.acl_classify(keys)
    finally:
        nf.close()
    for f in ("rule", "action", "scope", "acl"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert len(bad) == 0, f"{f}: {len(bad)} keys differ, first {keys[bad[0]]}: {got[bad[0]]} vs {want[bad[0]]}"
    h = {int(c): int((want["acl"] == c).sum()) for c in np.unique(want["acl"])}
    assert h.get(1, 0) and h.get(2, 0) and h.get(0, 0), h


def as_key(k) -> bytes:
    """AclKey::as_key (acl-filter/src/context.rs:168-190 through
    match-action-derive/src/lib.rs:191-206, 341-347): proto (NextHeader, 1 B),
    src_vni and dst_vni (Vni: 4 B, net/src/fixed_size.rs:61-74), the two
    addresses, the two ports -- every field big-endian, back to back."""
    al = 4 if int(k["family"]) == 4 else 16
    return (struct.pack(">BII", int(k["proto"]), int(k["src_vni"]), int(k["dst_vni"])) +
            bytes(k["src"][:al]) + bytes(k["dst"][:al]) + struct.pack(">HH", int(k["sport"]), int(k["dport"])))


def match_keys(keys: np.ndarray, fam: int, stride: int = 0) -> tuple:
    sel = keys[keys["family"] == fam]
    size = A.ACL_MATCH_KEY_V4 if fam == 4 else A.ACL_MATCH_KEY_V6
    stride = stride or size
    buf = np.zeros(len(sel) * stride, np.uint8)
    for i, k in enumerate(sel):
        buf[i * stride:i * stride + size] = np.frombuffer(as_key(k), np.uint8)
    return sel, buf, size, stride


@pytest.mark.parametrize("stride", [0, 64])
def test_acl_key_from_match(stride):
    import ctypes as C
    lib = A.gpu_lib()  # (host code of the library: no device is touched)
    r = np.random.default_rng(7 + stride)
    n = 500
    keys = np.zeros(n, A.ACL_KEY)
    keys["family"] = np.where(r.random(n) < 0.5, 4, 6)
    keys["proto"] = r.choice([1, 6, 17, 58], n)
    keys["src_vni"] = r.integers(1, 1 << 24, n)
    keys["dst_vni"] = r.integers(1, 1 << 24, n)
    keys["sport"] = r.integers(0, 65536, n)
    keys["dport"] = r.integers(0, 65536, n)
    keys["src"] = r.integers(0, 256, (n, 16))
    keys["dst"] = r.integers(0, 256, (n, 16))
    keys["src"][keys["family"] == 4, 4:] = 0
    keys["dst"][keys["family"] == 4, 4:] = 0
    for fam in (4, 6):
        sel, buf, size, st = match_keys(keys, fam, stride)
        assert len(buf) == len(sel) * st and size == (21 if fam == 4 else 45)
        got = np.zeros(len(sel), A.ACL_KEY)
        assert lib.dp_acl_key_from_match(buf.ctypes.data, size, st, len(sel), got.ctypes.data) == 0
        assert got.tobytes() == sel.tobytes()
    out = np.zeros(1, A.ACL_KEY)
    buf = np.zeros(64, np.uint8)
    assert lib.dp_acl_key_from_match(buf.ctypes.data, 20, 20, 1, out.ctypes.data) == -22  # DP_EINVAL
    assert lib.dp_acl_key_from_match(buf.ctypes.data, 21, 20, 1, out.ctypes.data) == -22  # DP_EINVAL
    assert lib.dp_acl_key_from_match(C.c_void_p(0), 45, 45, 0, C.c_void_p(0)) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [2, 5])
def test_gpu_acl_classify_match_10k(cfg):
    """BASELINE's ACL size (10k rules) through the reference's key bytes:
    dp_acl_classify_match == dp_acl_classify == the oracle, per family."""
    from dataplane_amd import GpuPathNf
    w = Workload(cfg, 20000, seed=90 + cfg, n_routes_v4=4000, n_routes_v6=2000, n_acl=10000, n_nat=16)
    o = Oracle(w.tables)
    res = o.process(w.fresh_buf(), w.inp)
    _, keys = keys_of(w, res, res)
    keys = np.concatenate([keys, perturb(keys, 10 + cfg)])
    keys = keys[np.isin(keys["family"], [4, 6])]
    want = o.acl_classify(keys)
    nf = GpuPathNf(0)
    try:
        nf.publish(w.tables)
        direct = nf.acl_classify(keys)
        for fam in ((4, 6) if cfg == 5 else (4,)):
            sel, buf, size, st = match_keys(keys, fam, 48)
            got = nf.acl_classify_match(buf, size, st)
            m = keys["family"] == fam
            for f in ("rule", "action", "scope", "acl"):
                assert np.array_equal(got[f], want[f][m]), (fam, f)
                assert np.array_equal(direct[f][m], want[f][m]), (fam, f)
    finally:
        nf.close()
    h = {int(c): int((want["acl"] == c).sum()) for c in np.unique(want["acl"])}
    assert h.get(1, 0) and h.get(2, 0), h
