"""CPU: the multi-GPU path's split -> process -> merge under gloo, world size
2 and 3.  Rank 0 holds a burst; scatter_burst moves each rank its byte span
and rebased in-records with grouped point-to-point sends (the calls the nccl
backend runs as RCCL over xGMI), every rank processes its shard (the oracle
stands in for the HIP path here), gather_burst brings the rewritten spans and
out-records back, and the merged result must equal one single-rank run of the
whole burst bit for bit.  Also: the bench's max-over-ranks timing and summed
DoneReason histogram."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, layout, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dataplane_amd import _abi as A
    from dataplane_amd import shard as SH
    from dataplane_amd.workload import Workload
    from oracle.pyoracle import Oracle
    # every rank builds the same tables (replicated per GPU); rank 0 owns the burst
    w = Workload(2, 3001, seed=7, n_routes_v4=3000, n_acl=200, n_nat=16, tcp_percent=30,
                 layout=layout)
    orc = Oracle(w.tables)
    shards = SH.split_burst(w.inp, w.buf.nbytes, world)
    dev = torch.device("cpu")
    buf = torch.from_numpy(w.fresh_buf())
    inp_u8 = torch.from_numpy(w.inp.view(np.uint8).copy())
    span, rin = SH.scatter_burst(buf, inp_u8, shards, A.PKT_IN.itemsize, rank, world, dev)
    s = shards[rank]
    sb = span.numpy()
    out = np.zeros(max(1, s.cnt), dtype=A.PKT_RES)
    if s.cnt:
        out = orc.process(sb, rin.numpy()[:s.cnt * A.PKT_IN.itemsize].view(A.PKT_IN))
    out_all = torch.zeros(w.n * A.PKT_RES.itemsize, dtype=torch.uint8)
    SH.gather_burst(span, torch.from_numpy(out.view(np.uint8).copy()), buf, out_all, shards,
                    A.PKT_RES.itemsize, rank, world)
    hist = np.bincount(out["done"][:s.cnt], minlength=A.DONE_COUNT)[:A.DONE_COUNT]
    elapsed, total = SH.reduce_over_ranks(0.5 + rank, hist, "cpu")
    res = None
    if rank == 0:
        merged = SH.rebase_gathered(out_all.numpy().view(A.PKT_RES), shards)
        b_ref = w.fresh_buf()
        o_ref = orc.process(b_ref, w.inp)
        res = dict(out_equal=bool(np.array_equal(merged, o_ref)),
                   buf_equal=bool(np.array_equal(buf.numpy(), b_ref)),
                   total=total.tolist(), ref_hist=np.bincount(o_ref["done"], minlength=A.DONE_COUNT)
                   [:A.DONE_COUNT].tolist(), elapsed=elapsed,
                   spans=[(x.lo, x.hi) for x in shards])
    q.put((rank, res))
    orc.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,layout", [(2, "packed"), (3, "dpdk")])
def test_scatter_process_gather_matches_single_rank(world, layout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, layout, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    r0 = res[0]
    assert r0["out_equal"], "merged out-records differ from the single-rank run"
    assert r0["buf_equal"], "gathered buffer differs from the single-rank run"
    assert r0["total"] == r0["ref_hist"]        # summed histogram over ranks
    assert r0["elapsed"] == 0.5 + world - 1     # max over ranks
    spans = r0["spans"]
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))  # disjoint spans


def test_split_rejects_overlapping_slots():
    from dataplane_amd import _abi as A
    from dataplane_amd import shard as SH
    inp = np.zeros(2, dtype=A.PKT_IN)
    inp["off"] = [96, 120]
    inp["len"] = [60, 60]
    with pytest.raises(ValueError):
        SH.split_burst(inp, 4096, 2)


def _timed_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dataplane_amd import _abi as A
    from dataplane_amd import shard as SH
    from dataplane_amd.workload import Workload
    from oracle.pyoracle import Oracle
    w = Workload(2, 2000, seed=9, n_routes_v4=2000, n_acl=100, n_nat=8, layout="dpdk")
    orc = Oracle(w.tables)

    def process(span, rin, cnt):
        out = np.zeros(max(1, cnt), dtype=A.PKT_RES)
        if cnt:
            out = orc.process(span.numpy(), rin.numpy()[:cnt * A.PKT_IN.itemsize].view(A.PKT_IN))
        return torch.from_numpy(out.view(np.uint8).copy())
    res = SH.timed_scatter_gather(w.inp, w.fresh_buf, process, rank, world, torch.device("cpu"),
                                  A.PKT_IN.itemsize, A.PKT_RES.itemsize, reps=2)
    q.put((rank, res))
    orc.close()
    dist.destroy_process_group()


def test_timed_scatter_gather_reports_on_root():
    """bench.py's N > 1 resident-burst measurement (scatter, per-rank
    processing, gather) runs to completion on every rank and reports the
    phases and link bytes on the root."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_timed_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    r0, r1 = res[0], res[1]
    assert r1 == {}
    assert r0["ranks"] == 2 and r0["packets"] == 2000
    assert r0["scatter_bytes"] > 1000 * 64 and r0["gather_bytes"] > 1000 * 64
    assert r0["scatter_ms"] >= 0 and r0["gather_ms"] >= 0 and r0["process_ms"] > 0
