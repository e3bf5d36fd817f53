"""Experiment: how much does the order of a burst's packets (which packets
share a wave, a workgroup, an XCD, a moment) change dp_pipeline_kernel's
time on C2?  Same packets and frames, only the dp_pkt_in_t records are
permuted.  Orders: as generated (random), sorted by source VNI (at any moment
every XCD reads one VPC's tables), XCD-aligned by source VNI (workgroup b runs
on XCD b % 8; XCDs 2v, 2v+1 get VPC v), sorted by destination address (the
FIB's direct-table lines shared by neighbours)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from dataplane_amd import GpuPathNf, _abi as A  # noqa: E402
from dataplane_amd.workload import Workload  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    w = Workload(cfg, 2_000_000, seed=1, layout="dpdk")
    nf = GpuPathNf(0)
    nf.publish(w.tables)
    n = w.n
    inp = w.inp
    off = inp["off"].astype(np.int64)
    dst = (w.buf[off + 30].astype(np.uint32) << 24) | (w.buf[off + 31].astype(np.uint32) << 16) | \
          (w.buf[off + 32].astype(np.uint32) << 8) | w.buf[off + 33].astype(np.uint32)
    vni = inp["src_vni"].astype(np.int64)
    orders = {"generated": np.arange(n)}
    rng = np.random.default_rng(7)
    orders["shuffled"] = rng.permutation(n)
    orders["by_src_vni"] = np.argsort(vni, kind="stable")
    # XCD-aligned: workgroup b (128 packets) takes its packets from VNI group (b % 8) * G // 8
    groups = [np.nonzero(vni == v)[0] for v in np.unique(vni)]
    G = len(groups)
    ptr = [0] * G
    blocks = []
    b = 0
    while any(p < len(g) for g, p in zip(groups, ptr)):
        gi = (b % 8) * G // 8
        for k in range(G):  # the preferred group, else the next non-empty one
            j = (gi + k) % G
            if ptr[j] < len(groups[j]):
                blocks.append(groups[j][ptr[j]:ptr[j] + 128])
                ptr[j] += 128
                break
        b += 1
    orders["xcd_src_vni"] = np.concatenate(blocks)
    orders["by_dst"] = np.argsort(dst, kind="stable")
    # sorted by destination, each XCD on its own eighth of the sorted order:
    # workgroup b takes the next 128 packets of part b % 8
    srt = np.argsort(dst, kind="stable")
    parts = np.array_split(srt, 8)
    pos8 = [0] * 8
    xb = []
    b = 0
    while any(p < len(q) for q, p in zip(parts, pos8)):
        j = b % 8
        if pos8[j] < len(parts[j]):
            xb.append(parts[j][pos8[j]:pos8[j] + 128])
            pos8[j] += 128
        else:
            xb.append(np.zeros(0, dtype=srt.dtype))  # keep the XCD rotation
        b += 1
    orders["xcd_dst"] = np.concatenate(xb)
    # source VNI, then the destination's top 8 bits within it
    orders["by_vni_dst8"] = np.lexsort((dst >> 24, vni))
    # coarse destination buckets (a device counting sort's key): top 8 / 12 / 16 bits,
    # packets of one bucket in burst order
    for b in (8, 12, 16):
        orders[f"by_dst{b}"] = np.argsort(dst >> (32 - b), kind="stable")
    only = os.environ.get("ORDERS")
    if only:
        orders = {k: v for k, v in orders.items() if k in only.split(",")}
    bb = (w.buf.nbytes + 255) & ~255
    pristine = torch.from_numpy(w.buf).to(dev)
    buf = torch.empty(bb, dtype=torch.uint8, device=dev)
    dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    res = {}
    for name, perm in orders.items():
        assert len(perm) == n and len(np.unique(perm)) == n
        dinp = torch.from_numpy(inp[perm].view(np.uint8).copy()).to(dev)
        ts = []
        for r in range(25):
            buf[:w.buf.nbytes].copy_(pristine)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            e0.record(stream)
            nf.process_device(buf.data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n, None,
                              stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            if r >= 5:
                ts.append(e0.elapsed_time(e1))
        res[name] = sorted(ts)[len(ts) // 2]
        print(f"C{cfg} {name:12s} kernel {res[name]:.4f} ms  {n / res[name] / 1e3:.0f} Mpps", flush=True)
    nf.close()


if __name__ == "__main__":
    main()
