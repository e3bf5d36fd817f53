# SPDX-License-Identifier: Apache-2.0
"""Multi-GPU sharding of the packet path.

Packets are independent, so N GPUs process N disjoint shards with no
data-path collective.  The only cross-rank steps are the bench's timing
(max over ranks) and the DoneReason histogram (sum over ranks), done with
torch.distributed (RCCL on GPUs, gloo in the CPU tests).
"""
from __future__ import annotations

import numpy as np


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
