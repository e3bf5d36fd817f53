"""A/B: dp_pipeline_kernel with the context tables in a per-workgroup LDS
copy (parts 1 / 2) against reading them from HBM (parts 11 / 12,
dpf_debug_no_ctx), alternating rounds of launches on one box.

    python scripts/probe/ctx_ab.py 2
"""
import os
import sys

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
    lib = A.gpu_lib()
    n = w.n
    bb = (w.buf.nbytes + 255) & ~255
    pristine = torch.from_numpy(w.buf).to(dev)
    buf = torch.empty(bb, dtype=torch.uint8, device=dev)
    dinp = torch.from_numpy(w.inp.view(np.uint8).copy()).to(dev)
    dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(dev)
    res = {"lds": [], "hbm": []}
    outs = {}
    for rnd in range(6):
        for name in ("lds", "hbm"):
            lib.dpf_debug_no_ctx(1 if name == "hbm" else 0)
            for r in range(8):
                buf[:w.buf.nbytes].copy_(pristine)
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                nf.process_device(buf.data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n, None, stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                if r >= 2:
                    res[name].append(e0.elapsed_time(e1))
            outs[name] = (dout.cpu().numpy().copy(), buf[:w.buf.nbytes].cpu().numpy().copy())
    lib.dpf_debug_no_ctx(0)
    same = all(np.array_equal(a, b) for a, b in zip(outs["lds"], outs["hbm"]))
    for k, v in res.items():
        m = sorted(v)[len(v) // 2]
        print(f"C{cfg} {k}: median {m:.4f} ms  {n / m / 1e3:.0f} Mpps  ({len(v)} launches)")
    print(f"C{cfg} outputs identical: {same}")
    nf.close()


if __name__ == "__main__":
    main()
