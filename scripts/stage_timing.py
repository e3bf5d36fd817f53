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

STAGES = ["window", "parse", "ingress/ipf1/seed", "icmp+flowfilter", "acl", "nat", "ipf2",
          "egress", "serialize+out"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--packets", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--acl", type=int, default=0)
    ap.add_argument("--nat", type=int, default=0)
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
    for r in range(a.reps + 1):
        db[:w.buf.nbytes].copy_(pristine)
        torch.cuda.synchronize()
        if r == 1:
            lib.dp_debug_stage_cycles(cyc.ctypes.data, 1)
        nf.process_device(db.data_ptr(), bb, di.data_ptr(), do.data_ptr(), w.n, None, s.cuda_stream)
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
    print(json.dumps({"config": a.config, "acl": a.acl, "nat": a.nat, "stages": res,
                      "wave_trips": trips}))


if __name__ == "__main__":
    main()
