"""GPU: the flow-filter classifier alone through the C ABI (dp_ff_classify,
dp_ff_classify_match) against the oracle -- the reference's context KATs
(tests/golden/ffkat.py), the workloads' flow-filter tables with the packets'
own lookups and perturbed ones, and a synthetic 10k-rule table per stage
(BASELINE's classifier size) over both classifier forms, v4 and v6, through
LookupInput records and through the reference's RemoteKey / LocalKey bytes."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from dataplane_amd.tables import TablesBuilder as TB
from golden import ffkat
from oracle.pyoracle import Oracle
from test_ff_classify import ff_inputs_of, local_key, match_buf, remote_key

pytestmark = pytest.mark.gpu
FIELDS = ("outcome", "dst_nat", "src_nat", "dst_vni")


@pytest.fixture(scope="module", autouse=True)
def torch_first():
    import torch
    torch.cuda.init()


def same(got, want, what):
    for f in FIELDS:
        bad = np.nonzero(got[f] != want[f])[0]
        assert len(bad) == 0, f"{what}: {f} differs for {len(bad)}, first {bad[0]}: {got[bad[0]]} vs {want[bad[0]]}"


@pytest.mark.parametrize("form", ["list", "bv"])
def test_gpu_ff_kat(form, cls_form):
    from dataplane_amd import GpuPathNf
    cls_form(A.gpu_lib(), form)
    for case in ffkat.cases():
        t = ffkat.tables(case)
        q = ffkat.inputs(case.probes)
        o = Oracle(t.build())
        want = o.ff_classify(q)
        o.close()
        nf = GpuPathNf(0)
        try:
            nf.publish(t.build())
            got = nf.ff_classify(q)
        finally:
            nf.close()
        errs = ffkat.check(case, got)
        assert not errs, "\n".join(errs)
        same(got, want, case.name)


def perturb(q: np.ndarray, seed: int) -> np.ndarray:
    r = np.random.default_rng(seed)
    k = q.copy()
    n = len(k)
    k["sport"] = np.where(r.random(n) < 0.4, r.integers(0, 65536, n), k["sport"])
    k["dport"] = np.where(r.random(n) < 0.4, r.integers(0, 65536, n), k["dport"])
    flip = r.random(n) < 0.3
    k["dst"][flip, 2] ^= r.integers(1, 256, int(flip.sum())).astype(np.uint8)
    flip = r.random(n) < 0.3
    k["src"][flip, 1] ^= r.integers(1, 256, int(flip.sum())).astype(np.uint8)
    k["gate"] = (r.random(n) < 0.1).astype(np.uint8)
    gated = r.random(n) < 0.1
    k["dst_vni"][gated] = k["src_vni"][np.roll(np.arange(n), 1)][gated]
    odd = r.random(n) < 0.02
    k["dst_family"][odd] = 10 - k["dst_family"][odd]  # a version mismatch
    return k


@pytest.mark.parametrize("cfg", [2, 5])
@pytest.mark.parametrize("form", ["list", "bv"])
def test_gpu_ff_classify_workload(cfg, form, cls_form):
    from dataplane_amd import GpuPathNf
    from dataplane_amd.workload import Workload
    w = Workload(cfg, 20000, seed=60 + cfg, n_routes_v4=4000, n_routes_v6=2000, n_acl=600, n_nat=16)
    o = Oracle(w.tables)
    res = o.process(w.fresh_buf(), w.inp)
    _, q = ff_inputs_of(w, res)
    q = np.concatenate([q, perturb(q, cfg)])
    want = o.ff_classify(q)
    o.close()
    cls_form(A.gpu_lib(), form)
    nf = GpuPathNf(0)
    try:
        nf.publish(w.tables)
        got = nf.ff_classify(q)
    finally:
        nf.close()
    same(got, want, f"C{cfg} {form}")
    h = np.bincount(want["outcome"], minlength=3)
    assert h.min() > 0, h


def rules_10k(seed: int):
    """10k remote and 10k local rules per family over 64 VPCs: prefixes of
    every length inside a few /8s (v4) and 2001:db8::/32 (v6), port ranges,
    protocols, gated masquerade destinations, PortFwdReply-gated sources, NAT
    modes; priorities by prefix length, the port-forwarding tie bit."""
    r = np.random.default_rng(seed)
    t = TB()
    t.add_iface(1, "02:00:00:00:00:01")
    vnis = [100 + 7 * k for k in range(64)]
    for v in vnis:
        t.add_fib(v, vnis=[v])
    def pfx(fam):
        if fam == 4:
            ln = int(r.integers(8, 33))
            a = (int(r.choice([10, 20, 30, 40])) << 24) | int(r.integers(0, 1 << 24))
            a &= ~((1 << (32 - ln)) - 1) & 0xffffffff
            return f"{a >> 24}.{a >> 16 & 255}.{a >> 8 & 255}.{a & 255}/{ln}"
        ln = int(r.integers(32, 129))
        import ipaddress
        a = (0x20010db8 << 96) | int(r.integers(0, 1 << 62)) << 34 | int(r.integers(0, 1 << 34))
        a &= ~((1 << (128 - ln)) - 1)
        return f"{ipaddress.IPv6Address(a)}/{ln}"
    def ports():
        x = r.random()
        if x < 0.6:
            return (0, 65535)
        lo = int(r.integers(1, 65000))
        return (lo, lo + int(r.integers(0, 500)))
    for fam in (4, 6):
        for _ in range(10_000):
            s, d = int(r.choice(vnis)), int(r.choice(vnis))
            mode = int(r.choice([0, 0, 1, 2, 3]))
            proto = [None, 6, 17][int(r.integers(0, 3))]
            t.add_ff_remote(s, pfx(fam), d, mode, proto=proto, dports=ports(),
                            gate_vni=d if mode == 2 else 0, port_forwarding=mode == 3)
            t.add_ff_local(s, d, pfx(fam), mode, proto=proto, sports=ports(), gate=1 if mode == 3 else 0)
    return t, vnis


def probes_for(t: TB, vnis, n: int, seed: int) -> np.ndarray:
    """Inputs aimed at the rules: an address inside a rule's prefix (or near
    it), the rule's VPCs, ports inside or outside its range."""
    r = np.random.default_rng(seed)
    q = np.zeros(n, A.FF_INPUT)
    rem = t.ff_remote[4] + t.ff_remote[6]
    loc = t.ff_local[4] + t.ff_local[6]
    for i in range(n):
        j = int(r.integers(0, len(rem)))
        a = rem[j]  # (the local rule added with it: its peering)
        b = loc[j] if r.random() < 0.8 else loc[int(r.integers(0, len(loc)))]
        fam = a.family if r.random() < 0.9 else b.family
        al = 4 if fam == 4 else 16
        q[i]["src_family"] = q[i]["dst_family"] = fam
        q[i]["src_vni"] = a.vni_a if r.random() < 0.9 else int(r.choice(vnis))
        q[i]["dst_vni"] = a.vni_b if r.random() < 0.5 else 0
        q[i]["proto"] = int(r.choice([6, 17, 1, a.proto_val or 6]))
        q[i]["gate"] = int(r.random() < 0.3)
        q[i]["dport"] = int(r.integers(a.dport_lo, a.dport_hi + 1)) if r.random() < 0.8 else int(r.integers(0, 65536))
        q[i]["sport"] = int(r.integers(b.sport_lo, b.sport_hi + 1)) if r.random() < 0.8 else int(r.integers(0, 65536))
        for f, rule, pf in (("dst", a, a.dst), ("src", b, b.src)):
            addr = bytes(pf.addr)[:al] if pf.family == fam else bytes(r.integers(0, 256, al, dtype=np.uint8))
            x = bytearray(addr)
            host = al * 8 - (pf.len if pf.family == fam else 0)
            for bit in range(host):  # random host bits inside the prefix
                if r.random() < 0.5:
                    x[al - 1 - bit // 8] ^= 1 << (bit % 8)
            if r.random() < 0.1:
                x[int(r.integers(0, al))] ^= 0x10  # outside, now and then
            q[i][f][:al] = np.frombuffer(bytes(x), np.uint8)
    return q


@pytest.mark.parametrize("form", ["list", "bv"])
def test_gpu_ff_classify_10k(form, cls_form):
    from dataplane_amd import GpuPathNf
    t, vnis = rules_10k(3)
    q = probes_for(t, vnis, 30_000, 4)
    o = Oracle(t.build())
    want = o.ff_classify(q)
    want1 = o.ff_classify(q, stage=1)
    q2 = q.copy()
    q2["dst_vni"] = np.where(want["outcome"] != 0, want["dst_vni"], q["dst_vni"])
    want2 = o.ff_classify(q2, stage=2)
    o.close()
    h = np.bincount(want["outcome"], minlength=3)
    assert h.min() > 1000, h
    cls_form(A.gpu_lib(), form)
    nf = GpuPathNf(0)
    try:
        nf.publish(t.build())
        got = nf.ff_classify(q)
        same(got, want, f"10k {form}")
        # the two tables alone over the reference's key bytes
        for fam in (4, 6):
            m = q["src_family"] == fam
            g1 = nf.ff_classify_match(A.FF_REMOTE, match_buf([remote_key(k) for k in q[m]], 32),
                                      A.FF_REMOTE_KEY_V4 if fam == 4 else A.FF_REMOTE_KEY_V6, 32)
            same(g1, want1[m], f"10k {form} remote v{fam}")
            g2 = nf.ff_classify_match(A.FF_LOCAL, match_buf([local_key(k) for k in q2[m]], 32),
                                      A.FF_LOCAL_KEY_V4 if fam == 4 else A.FF_LOCAL_KEY_V6, 32)
            same(g2, want2[m], f"10k {form} local v{fam}")
    finally:
        nf.close()
