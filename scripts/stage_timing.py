"""Per-stage wave time of dp_pipeline_kernel (diagnostic build with -DDP_TIMING).

    DPGPU_LIB=dataplane_amd/lib/libdpgpu_timing.so python scripts/stage_timing.py --config 2
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("DPGPU_LIB", os.path.join(ROOT, "dataplane_amd/lib/libdpgpu_timing.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dataplane_amd import GpuPathNf, _abi as A  # noqa: E402
from dataplane_amd.workload import Workload  # noqa: E402

STAGES = ["window", "parse", "ingress/ipf1/seed", "flowfilter", "acl", "nat", "ipf2",
          "egress", "serialize+out", "icmp+flowlookup"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--packets", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--acl", type=int, default=0)
    ap.add_argument("--nat", type=int, default=0)
    ap.add_argument("--flows", action="store_true",
                    help="a flow table attached, every other packet's flow pair established (bench.py flows_leg)")
    ap.add_argument("--meta", action="store_true", help="meta records written")
    a = ap.parse_args()
    torch.cuda.init()
    dev = torch.device("cuda", 0)
    w = Workload(a.config, a.packets, seed=1, n_acl=a.acl, n_nat=a.nat, layout="dpdk")
    nf = GpuPathNf(0)
    nf.publish(w.tables)
    lib = A.gpu_lib()
    lib.dp_debug_stage_cycles.argtypes = [C.c_void_p, C.c_int]
    cyc = np.zeros(16, dtype=np.uint64)
    bb = (w.buf.nbytes + 255) & ~255
    pristine = torch.from_numpy(w.buf).to(dev)
    db = torch.empty(bb, dtype=torch.uint8, device=dev)
    di = torch.from_numpy(w.inp.view(np.uint8)).to(dev)
    do = torch.empty(w.n * 32, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    dm = torch.empty(w.n * A.PKT_META.itemsize, dtype=torch.uint8, device=dev)
    mkw = {"dev_meta": dm.data_ptr()} if (a.meta or a.flows) else {}
    ft = None
    if a.flows:
        from dataplane_amd.flows import FlowTable, burst_request_flows
        db[:w.buf.nbytes].copy_(pristine)
        nf.process_device(db.data_ptr(), bb, di.data_ptr(), do.data_ptr(), w.n, None, s.cuda_stream,
                          dev_meta=dm.data_ptr())
        s.synchronize()
        meta = dm.cpu().numpy().view(A.PKT_META)
        fl = burst_request_flows(w.buf, w.inp, np.arange(0, w.n, 2), meta["dst_vni"], nf.data.genid)
        ft = FlowTable(0, 1 << max(12, int(np.ceil(np.log2(max(1, 4 * len(fl)))))))
        ft.set_capacity(len(fl))
        ft.insert(fl)
        nf.attach_flows(ft)
    for r in range(a.reps + 1):
        db[:w.buf.nbytes].copy_(pristine)
        torch.cuda.synchronize()
        if r == 1:
            lib.dp_debug_stage_cycles(cyc.ctypes.data, 1)
        nf.process_device(db.data_ptr(), bb, di.data_ptr(), do.data_ptr(), w.n, None, s.cuda_stream, **mkw)
        s.synchronize()
    lib.dp_debug_stage_cycles(cyc.ctypes.data, 0)
    tot = float(cyc[:len(STAGES)].sum())
    res = {k: round(float(cyc[i]) / tot, 4) for i, k in enumerate(STAGES)}
    waves = a.reps * ((w.n + 63) // 64)
    res["cycles_per_wave"] = round(tot / waves, 1)
    # -DDP_GPU_TRIPS builds: wave-level loop iterations per wave
    trips = {k: round(float(cyc[i]) / waves, 3) for i, k in
             [(12, "indexed_verify_calls"), (13, "ff_verify_iters"), (14, "acl_verify_iters"),
              (15, "hoisted_verify_calls")]}
    if ft is not None:
        nf.attach_flows(None)
        ft.close()
    print(json.dumps({"config": a.config, "acl": a.acl, "nat": a.nat, "flows": a.flows, "meta": a.meta,
                      "stages": res,
                      "wave_trips": trips}))


if __name__ == "__main__":
    main()
