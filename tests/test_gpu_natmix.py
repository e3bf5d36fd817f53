"""GPU: bursts that mix port forwarding and masquerade on one public range
(the reference's overlapping-expose configuration, nat/src/test.rs:141-174,
scaled up as dataplane_amd/natwork.py mixed_world), bit-exact against the
oracle: every record, the whole buffer, both flows of every connection by key
and the flow counts.

The NAT pass runs such a burst in mode 5 -- the port-forwarding connections as
lanes beside the masquerade split -- and falls back to the one-lane pass where
the two parts could meet: a forwarded host answering in the
very burst that opens its connection (its packet masquerades on the key the
creation inserts, dp_nat_cross), a table without room for every pair."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from dataplane_amd import natwork as W
from golden.masqkat import GpuRunner, OracleRunner
from helpers import hist
from test_gpu_nat_scale import both, same_flows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def torch_first():
    import torch
    torch.cuda.init()


@pytest.mark.parametrize("e,n,force,fork", [(2_000, 20_000, 0, 2), (2_000, 20_000, 0, 3), (2_000, 20_000, 4, 2),
                                            (125_000, 300_000, 0, 2)],
                         ids=["small", "small-steady-replay-early", "small-no-mode5", "250k-connections"])
def test_gpu_mixed_bursts(e, n, force, fork):
    """fork: where the replay leaves for the side stream (dpf_debug_replay_fork:
    2 after the lane's plan, 3 the steady refreshes right after dp_nat_prep)."""
    ro, rg = OracleRunner(), GpuRunner(slots=1 << 22)
    A.gpu_lib().dpf_debug_nat_sequential(force)
    A.gpu_lib().dpf_debug_replay_fork(fork)
    want = 1 if force == 4 else 5
    try:
        for r in (ro, rg):
            r.publish(W.mixed_world())
            r.set_clock(10 ** 12)
        c = W.MixedConns(e, e)
        buf, inp = c.first()
        out, ob, cnt = both(ro, rg, buf, inp, "first packets")
        assert hist(out) == {"Delivered": 2 * e}, hist(out)
        assert int(cnt[12]) == want, cnt
        assert c.learn(ob, out) == e
        assert not ((c.pport >= 3000) & (c.pport <= 3999)).any(), "a claimed port masqueraded"
        keys = c.keys()
        assert same_flows(ro, rg, keys, "first packets") == 2 * e
        # established on both sides (answers move the pairs two-way, then
        # established: steady refreshes), 2 % new connections of both kinds
        for step in (1, 2, 3):
            for r in (ro, rg):
                r.set_clock(10 ** 12 + step * 10 ** 9)
            buf, inp, npf, nm = c.burst(n, 0.02, step)
            out, ob, cnt = both(ro, rg, buf, inp, f"mixed burst {step}")
            assert hist(out) == {"Delivered": n}, hist(out)
            assert int(cnt[12]) == want, (step, cnt)
            if want == 5:
                assert int(cnt[4]) > 0 and int(cnt[11]) >= nm, cnt  # connection lanes; the allocating lane
            assert same_flows(ro, rg, keys, f"mixed burst {step}") == 2 * e
        if want == 5:
            assert int(cnt[27]) == 1, cnt  # steady refreshes in the last burst
        # forwarded hosts answering the new connections in the same burst:
        # one lane (and the same outcome)
        for r in (ro, rg):
            r.set_clock(10 ** 12 + 4 * 10 ** 9)
        buf, inp, npf, nm = c.burst(n, 0.02, 4, same_burst_replies=7)
        out, ob, cnt = both(ro, rg, buf, inp, "mixed burst with same-burst replies")
        assert int(cnt[12]) == 1, cnt
        if want == 5:
            # dp_nat_cross found the replies' initial keys among the creations'
            assert int(cnt[30]) == 1 and int(cnt[34]) >= 7, cnt
        assert same_flows(ro, rg, keys, "mixed burst with same-burst replies") == 2 * e
        # without room for every pair: one lane
        for r in (ro, rg):
            r.set_clock(10 ** 12 + 5 * 10 ** 9)
            (r.fl if hasattr(r, "fl") else r.ft).set_capacity(r.count()[0] + 100)
        buf, inp, npf, nm = c.burst(n, 0.02, 5)
        out, ob, cnt = both(ro, rg, buf, inp, "mixed burst near capacity")
        assert int(cnt[12]) == 1, cnt
        assert hist(out).get("FlowCapacityExceeded", 0) > 0, hist(out)
    finally:
        A.gpu_lib().dpf_debug_nat_sequential(0)
        A.gpu_lib().dpf_debug_replay_fork(-1)
        rg.close()
