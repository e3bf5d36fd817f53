"""CPU: the multi-GPU bench path's cross-rank logic under gloo, world size 2
(each rank: its own seeded shard, processed by the oracle; max-over-ranks
timing and summed DoneReason histogram)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dataplane_amd import _abi as A
    from dataplane_amd.shard import reduce_over_ranks, shard_seed
    from dataplane_amd.workload import Workload
    from oracle.pyoracle import Oracle
    w = Workload(2, 2000, seed=shard_seed(7, rank), n_routes_v4=2000, n_acl=100, n_nat=16)
    out = Oracle(w.tables).process(w.fresh_buf(), w.inp, A.PKT_OUT)
    hist = np.bincount(out["done"], minlength=A.DONE_COUNT)[:A.DONE_COUNT]
    elapsed, total = reduce_over_ranks(0.5 + rank, hist, "cpu")
    q.put((rank, elapsed, total.tolist(), hist.tolist(), int(w.inp["off"][:64].sum()),
           bytes(w.buf[:4096]).hex()))
    dist.destroy_process_group()


def test_two_rank_shards_and_reduction():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (r0, e0, t0, h0, _, b0), (r1, e1, t1, h1, _, b1) = res
    assert e0 == e1 == 1.5                       # max over ranks
    assert t0 == t1 == [a + b for a, b in zip(h0, h1)]
    assert sum(t0) == 4000
    assert b0 != b1                              # independent shards
