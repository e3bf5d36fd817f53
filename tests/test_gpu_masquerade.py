"""GPU: masquerade through the C ABI against the oracle
-- the reference's Masquerade tests (nat/src/masquerade/test.rs, as
tests/golden/masqkat.py scenarios) and seeded bursts (tests/masqgen.py), every
step compared bit-exactly: records, delivered bytes, the packet's flow
(FlowStatus, masquerade state, allocation, expiry, generation, idle
timeout), each connection's two flows by key and the flow counts."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from golden import masqkat
from helpers import common_fields

pytestmark = pytest.mark.gpu

INFO = ("status", "flags", "dst_vni", "genid", "expires_at", "pf", "masq", "masq_alloc", "pf_status",
        "pf_port", "pf_family", "pf_ip", "idle_timeout_s")


def same_info(io, ig, what: str):
    for k in INFO:
        assert np.array_equal(io[k], ig[k]), f"{what}: flow {k} {io[k]} != {ig[k]}"


@pytest.fixture(scope="module", autouse=True)
def torch_first():
    import torch
    torch.cuda.init()


@pytest.mark.parametrize("s", masqkat.scenarios(), ids=lambda s: s.name)
def test_gpu_masquerade_kat(s):
    steps_o, steps_g = [], []
    errs = masqkat.run_scenario(s, masqkat.OracleRunner(),
                                lambda i, res, buf, info: steps_o.append((res.copy(), buf.copy(), info)))
    assert not errs, errs
    g = masqkat.GpuRunner()
    try:
        errs = masqkat.run_scenario(s, g, lambda i, res, buf, info: steps_g.append(
            (res.copy(), buf.copy(), info)))
    finally:
        g.close()
    assert not errs, "\n".join(errs)
    assert len(steps_o) == len(steps_g)
    for i, ((ro, bo, io), (rg, bg, ig)) in enumerate(zip(steps_o, steps_g)):
        a, b = common_fields(ro, rg)
        assert np.array_equal(a, b), f"step {i}: records {a} != {b}"
        o = ro[0]
        if o["done"] == A.DONE["Delivered"]:
            assert bo[o["off"]:o["off"] + o["len"]].tobytes() == bg[o["off"]:o["off"] + o["len"]].tobytes(), \
                f"step {i}: frame"
        assert (io is None) == (ig is None), f"step {i}: flow attached"
        if io is not None:
            same_info(io, ig, f"step {i}")


# (dpf_debug_nat_sequential, dpf_debug_replay_fork): the split pass with the
# replay off the allocating lane forked after the lane's plan (the default),
# after the resolve, the steady refreshes after dp_nat_prep, or not forked (one
# replay after the lane)
NAT_MODES = {"split": (0, 2), "split-fork-resolve": (0, 1), "split-fork-prep": (0, 3), "split-no-fork": (0, 0),
             "one-lane": (1, 2),
             "split-alone": (2, 2), "split-steps": (5, 2)}


@pytest.mark.parametrize("nat", list(NAT_MODES))
@pytest.mark.parametrize("seed,n_conn,capacity", [(1, 600, None), (2, 3000, None), (3, 800, 500)])
def test_gpu_masquerade_random_bursts(seed, n_conn, capacity, nat):
    """Seeded bursts (tests/masqgen.py): allocations from a shared, claimed
    public range until it runs out, repeats, replies, TCP handshakes /
    teardowns / resets, DNS answers, ICMP echo, uncovered sources, sweeps that
    return tuples, a same-config republish, a narrowed config and none -- and,
    with a small capacity, pairs refused at capacity; GPU == oracle per burst.
    nat: the masquerading bursts' split pass (connection lanes + the
    allocating lane with wave batches), the same with every allocation alone,
    or the one-lane pass (the test hook dpf_debug_nat_sequential); the replay
    of the records off the allocating lane beside it (forked at either point)
    or after it (dpf_debug_replay_fork)."""
    import masqgen
    from golden.masqkat import GpuRunner, OracleRunner
    got, modes = {}, []
    for name, mk in (("oracle", OracleRunner), ("gpu", GpuRunner)):
        r = mk(slots=1 << 15) if name == "gpu" else mk()
        steps = []

        def on(k, res, buf, infos, look, rel, pkts):
            steps.append((res.copy(), buf.copy(), infos.copy(), look.copy(), rel.copy(), r.count()))
            if name == "gpu":
                modes.append(r.nat_counters())
        if name == "gpu":
            A.gpu_lib().dpf_debug_nat_sequential(NAT_MODES[nat][0])
            A.gpu_lib().dpf_debug_replay_fork(NAT_MODES[nat][1])
        try:
            masqgen.run(r, seed, n_conn, capacity, on)
        finally:
            if name == "gpu":
                A.gpu_lib().dpf_debug_nat_sequential(0)
                A.gpu_lib().dpf_debug_replay_fork(-1)
                r.close()
        got[name] = steps
    hist = {}
    for k, (o, g) in enumerate(zip(got["oracle"], got["gpu"])):
        (ro, bo, io, lo, xo, co), (rg, bg, ig, lg, xg, cg) = o, g
        a, b = common_fields(ro, rg)
        bad = np.nonzero(a != b)[0]
        assert len(bad) == 0, f"burst {k}: {len(bad)} records differ, first {a[bad[0]]} vs {b[bad[0]]}"
        for i in np.nonzero(ro["done"] == A.DONE["Delivered"])[0]:
            s0, n0 = int(ro[i]["off"]), int(ro[i]["len"])
            assert np.array_equal(bo[s0:s0 + n0], bg[s0:s0 + n0]), f"burst {k} packet {i}: frame"
        same_info(io, ig, f"burst {k}: packets'")
        assert np.array_equal(lo["ref"] == A.FLOW_NONE, lg["ref"] == A.FLOW_NONE), f"burst {k}: presence"
        same_info(lo, lg, f"burst {k}: flows by key:")
        assert np.array_equal(xo["ref"] == A.FLOW_NONE, xg["ref"] == A.FLOW_NONE), f"burst {k}: related presence"
        same_info(xo, xg, f"burst {k}: related flows:")
        assert co == cg, f"burst {k}: counts {co} vs {cg}"
        for d in ro["done"]:
            hist[A.DONE_NAMES[d]] = hist.get(A.DONE_NAMES[d], 0) + 1
    assert hist.get("Delivered", 0) > n_conn
    ran = [int(c[12]) for c in modes]
    assert all(int(c[16]) == 0 for c in modes), "split pass refused a pair"
    if nat == "one-lane":
        assert set(ran) <= {0, 1}, ran
    else:
        # the masquerading bursts ran split: connection lanes and the
        # allocating lane, its allocations in wave batches or alone -- or,
        # with a small capacity (no room for every pair it could create),
        # its records one by one in packet order
        assert ran.count(3) >= 4, ran
        assert sum(int(c[11]) for c in modes) > 0
        if capacity is not None:
            assert any(int(c[18]) == int(c[11]) > 0 for c in modes)
        elif nat != "split-alone":
            assert sum(int(c[14]) for c in modes) > 0
            # (these bursts mix closes, resets and repeats into the lane: the
            # bulk serve rarely qualifies -- test_gpu_nat_scale covers it;
            # with it off, the lane's steps serve every allocation)
            if nat == "split-steps":
                assert sum(int(c[39]) for c in modes) == 0
        else:
            assert sum(int(c[14]) for c in modes) == 0 and sum(int(c[15]) for c in modes) > 0
    if n_conn >= 3000:
        assert hist.get("NatOutOfResources", 0) > 0
    if capacity is not None:
        assert hist.get("FlowCapacityExceeded", 0) > 0
