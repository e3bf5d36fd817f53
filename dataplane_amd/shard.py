# SPDX-License-Identifier: Apache-2.0
"""Multi-GPU sharding of the packet path.

Packets are independent (every stage is a per-packet function of the packet
and read-only tables), so a burst splits into contiguous shards of whole
packets that N GPUs process with no data-path dependency -- the analogue of
the reference's per-worker fan-out (``dataplane/src/drivers/kernel/fanout.rs:49-73``,
one pipeline per worker, ``worker.rs:175``).  Tables are replicated per GPU.

Three ways a burst reaches the GPUs:

- each rank owns its own shard from the start (bench weak scaling: no
  collective on the data path);
- host-origin bursts in one process: ``dp_process_burst_sharded`` (C ABI),
  one pinned ``hipMemcpyAsync`` per GPU;
- a burst resident on one GPU: ``scatter_burst`` / ``gather_burst`` move each
  rank's byte span and records with grouped point-to-point sends (RCCL over
  xGMI with the nccl backend; RCCL has no scatter primitive, and each peer
  gets its own link), and bring the rewritten spans and out-records back.

``split_burst`` / ``merge_outs`` are the pure split/merge arithmetic shared by
all three; the CPU tests run them under gloo (``tests/test_shard.py``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

HEADROOM = 96  # DP_HEADROOM: a packet owns [off - HEADROOM, off + len)


def shard_seed(seed: int, rank: int) -> int:
    """Every rank generates its own shard of the synthetic workload."""
    return seed + 1000 * rank


def reduce_over_ranks(elapsed_s: float, hist: np.ndarray, device) -> tuple:
    """(max elapsed over ranks, summed DoneReason histogram)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return elapsed_s, hist
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    h = torch.from_numpy(np.array(hist, dtype=np.int64)).to(device)  # a copy
    dist.all_reduce(h)
    return float(t.item()), h.cpu().numpy()


@dataclass
class Shard:
    """Packets [first, first + cnt) of a burst; their slots live in the byte
    span [lo, hi) of the burst buffer; `inp` holds their in-records with
    offsets relative to lo."""
    first: int
    cnt: int
    lo: int
    hi: int
    inp: np.ndarray


def shard_bounds(n: int, world: int) -> List[tuple]:
    """Shard k gets packets [k n / world, (k+1) n / world) (as the C ABI's
    dp_process_burst_sharded)."""
    return [(n * k // world, n * (k + 1) // world - n * k // world) for k in range(world)]


def split_burst(inp: np.ndarray, buf_bytes: int, world: int) -> List[Shard]:
    """Split a burst into `world` contiguous shards of whole packets.  The
    packets must be in buffer order with non-overlapping slots, so the
    shards' byte spans are disjoint."""
    off = inp["off"].astype(np.int64)
    ln = inp["len"].astype(np.int64)
    if len(inp) and (off.min() < HEADROOM or (off + ln).max() > buf_bytes or
                     np.any(off[1:] - HEADROOM < off[:-1] + ln[:-1])):
        raise ValueError("sharded bursts need in-order, non-overlapping packet slots")
    shards = []
    for first, cnt in shard_bounds(len(inp), world):
        if cnt == 0:
            shards.append(Shard(first, 0, 0, 0, inp[:0].copy()))
            continue
        # 64-byte aligned start (keeps DPDK-layout frames sector aligned on
        # the device), never below the previous packet's end: spans stay
        # disjoint, so concurrent write-backs never overlap
        prev_end = int(off[first - 1] + ln[first - 1]) if first else 0
        lo = max(prev_end, int(off[first] - HEADROOM) & ~63)
        hi = int(min(buf_bytes, off[first + cnt - 1] + ln[first + cnt - 1]))
        r = inp[first:first + cnt].copy()
        r["off"] = (off[first:first + cnt] - lo).astype(np.uint32)
        shards.append(Shard(first, cnt, lo, hi, r))
    return shards


def shard_buffer_bytes(s: Shard) -> int:
    """Bytes a rank allocates for a shard's span (frames are staged with
    16-byte loads past their end)."""
    return ((s.hi - s.lo + 15) & ~15) + 16


def merge_outs(shards: Sequence[Shard], outs: Sequence[np.ndarray]) -> np.ndarray:
    """Concatenate the shards' out-records with offsets back in the full
    burst's coordinates."""
    parts = []
    for s, o in zip(shards, outs):
        o = np.array(o[:s.cnt], copy=True)
        o["off"] = (o["off"].astype(np.int64) + s.lo).astype(np.uint32)
        parts.append(o)
    return np.concatenate(parts) if parts else np.zeros(0)


def _as_u8(t):
    import torch
    return t.view(torch.uint8) if t.dtype != torch.uint8 else t


def scatter_burst(buf, inp_u8, shards: Sequence[Shard], pkt_in_size: int, rank: int,
                  world: int, device, root: int = 0):
    """Move each rank's span of a burst held by `root` (torch uint8 tensors
    `buf`, `inp_u8` on `device`, only meaningful on the root) to that rank:
    grouped point-to-point sends from the root, one per peer (RCCL / gloo).
    Returns this rank's (span buffer, rebased in-records) tensors."""
    import torch
    import torch.distributed as dist
    s = shards[rank]
    span = torch.zeros(shard_buffer_bytes(s), dtype=torch.uint8, device=device)
    rin = torch.zeros(max(1, s.cnt) * pkt_in_size, dtype=torch.uint8, device=device)
    if rank == root:
        ops = []
        keep = []
        for k in range(world):
            sk = shards[k]
            if sk.cnt == 0:
                continue
            src_span = buf[sk.lo:sk.hi]
            src_in = torch.from_numpy(sk.inp.view(np.uint8)).to(device)
            keep += [src_span, src_in]
            if k == root:
                span[:sk.hi - sk.lo].copy_(src_span)
                rin[:src_in.numel()].copy_(src_in)
                continue
            ops.append(dist.P2POp(dist.isend, src_span.contiguous(), k))
            ops.append(dist.P2POp(dist.isend, src_in, k))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
    elif s.cnt:
        recv_span = torch.empty(s.hi - s.lo, dtype=torch.uint8, device=device)
        ops = [dist.P2POp(dist.irecv, recv_span, root),
               dist.P2POp(dist.irecv, rin[:s.cnt * pkt_in_size], root)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        span[:s.hi - s.lo].copy_(recv_span)
    return span, rin


def gather_burst(span, out_u8, buf, out_all_u8, shards: Sequence[Shard], pkt_out_size: int,
                 rank: int, world: int, root: int = 0) -> None:
    """Bring every rank's rewritten span and out-records back to the root
    (grouped point-to-point receives on the root), writing the spans into
    `buf` and the out-records (still span-relative) into `out_all_u8`."""
    import torch.distributed as dist
    s = shards[rank]
    if rank == root:
        ops = []
        for k in range(world):
            sk = shards[k]
            if sk.cnt == 0:
                continue
            dst_out = out_all_u8[sk.first * pkt_out_size:(sk.first + sk.cnt) * pkt_out_size]
            if k == root:
                buf[sk.lo:sk.hi].copy_(span[:sk.hi - sk.lo])
                dst_out.copy_(out_u8[:sk.cnt * pkt_out_size])
                continue
            ops.append(dist.P2POp(dist.irecv, buf[sk.lo:sk.hi], k))
            ops.append(dist.P2POp(dist.irecv, dst_out, k))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
    elif s.cnt:
        ops = [dist.P2POp(dist.isend, span[:s.hi - s.lo].contiguous(), root),
               dist.P2POp(dist.isend, out_u8[:s.cnt * pkt_out_size].contiguous(), root)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def rebase_gathered(out: np.ndarray, shards: Sequence[Shard]) -> np.ndarray:
    """Out-records gathered span-relative -> full-burst offsets."""
    out = out.copy()
    for s in shards:
        if s.cnt:
            o = out["off"][s.first:s.first + s.cnt].astype(np.int64) + s.lo
            out["off"][s.first:s.first + s.cnt] = o.astype(np.uint32)
    return out


def timed_scatter_gather(inp: np.ndarray, fresh_buf, process, rank: int, world: int, device,
                         pkt_in_size: int, pkt_out_size: int, reps: int = 3, root: int = 0) -> dict:
    """Cost of the resident-burst path on its own: the root's burst (`inp`,
    `fresh_buf()` -> its bytes) scattered to every rank, each shard processed
    there (`process(span, rin, cnt) -> out-records tensor`), spans and records
    gathered back.  Barrier-bracketed wall time of each phase, median over
    `reps` (after one untimed round); bytes are what crosses the links (the
    root's own shard is a local copy).  Returns the figures on the root."""
    import time

    import torch
    import torch.distributed as dist

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        dist.barrier()

    buf_np = fresh_buf() if rank == root else None
    buf_bytes = int(buf_np.nbytes) if rank == root else 0
    nb = torch.tensor([buf_bytes], dtype=torch.int64, device=device)
    dist.broadcast(nb, root)
    shards = split_burst(inp, int(nb.item()), world)
    buf = torch.from_numpy(buf_np).to(device) if rank == root else None
    inp_u8 = torch.from_numpy(inp.view(np.uint8).copy()).to(device) if rank == root else None
    out_all = (torch.empty(len(inp) * pkt_out_size, dtype=torch.uint8, device=device)
               if rank == root else None)
    times = []
    for r in range(reps + 1):
        sync()
        t0 = time.perf_counter()
        span, rin = scatter_burst(buf, inp_u8, shards, pkt_in_size, rank, world, device, root)
        sync()
        t1 = time.perf_counter()
        s = shards[rank]
        out = process(span, rin, s.cnt)
        sync()
        t2 = time.perf_counter()
        gather_burst(span, out, buf, out_all, shards, pkt_out_size, rank, world, root)
        sync()
        t3 = time.perf_counter()
        if r:
            times.append((t1 - t0, t2 - t1, t3 - t2))
    if rank != root:
        return {}
    med = [sorted(t[i] for t in times)[len(times) // 2] for i in range(3)]
    peers = [s for k, s in enumerate(shards) if k != root and s.cnt]
    sc_bytes = sum((s.hi - s.lo) + s.cnt * pkt_in_size for s in peers)
    ga_bytes = sum((s.hi - s.lo) + s.cnt * pkt_out_size for s in peers)
    return {"packets": int(len(inp)), "ranks": world,
            "scatter_ms": round(med[0] * 1e3, 3), "process_ms": round(med[1] * 1e3, 3),
            "gather_ms": round(med[2] * 1e3, 3),
            "scatter_bytes": int(sc_bytes), "gather_bytes": int(ga_bytes),
            "scatter_gbs": round(sc_bytes / med[0] / 1e9, 2) if med[0] else None,
            "gather_gbs": round(ga_bytes / med[2] / 1e9, 2) if med[2] else None,
            "mpps_end_to_end": round(len(inp) / sum(med) / 1e6, 2),
            "what": "a burst resident on the root GPU: grouped point-to-point sends of each "
                    "rank's byte span and records (RCCL over xGMI), per-rank processing, "
                    "gather back; barrier-bracketed phases, median of the timed rounds"}
