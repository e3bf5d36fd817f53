"""Chain-length model of dp_pipeline_kernel: dependent-load round trips per
packet and stage, from the host emulation built with -DDP_TRIPS
(tests/emu build/libdpemu_trips.so), and per wave of 64 consecutive packets
the sum over stages of the slowest lane's trips (lanes of a wave walk a
stage's loop in lockstep, so the wave waits for its longest chain).

    python scripts/trips.py --config 2 --packets 200000
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "emu"))

import numpy as np  # noqa: E402

from dataplane_amd import _abi as A  # noqa: E402
from dataplane_amd.workload import Workload  # noqa: E402

STAGES = ["-", "vni/ingress/ipf1", "ff remote", "pair+hoist+ff local", "acl", "nat", "ipf2", "egress"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--packets", type=int, default=200_000)
    ap.add_argument("--routes-v4", type=int, default=0)
    a = ap.parse_args()
    os.environ["DPEMU_LIB"] = os.path.join(ROOT, "tests/emu/build/libdpemu_trips.so")
    import pyemu
    lib = pyemu.lib()
    lib.dpemu_trips_out.argtypes = [C.c_void_p]
    w = Workload(a.config, a.packets, seed=1, n_routes_v4=a.routes_v4, layout="dpdk")
    trips = np.zeros((w.n, 8), dtype=np.uint16)
    lib.dpemu_trips_out(trips.ctypes.data)
    out = pyemu.process(w.tables, w.fresh_buf(), w.inp)
    lib.dpemu_trips_out(None)
    nw = w.n // 64
    t = trips[:nw * 64].reshape(nw, 64, 8).astype(np.int64)
    lane = t.mean(axis=(0, 1))
    wave = t.max(axis=1).mean(axis=0)
    print(f"C{a.config}: {w.n} packets; delivered {np.mean(out['done'] == A.DONE['Delivered']):.3f}")
    print(f"{'stage':24s} {'mean/lane':>10s} {'max-lane/wave':>14s}")
    for k in range(1, 8):
        print(f"{STAGES[k]:24s} {lane[k]:10.2f} {wave[k]:14.2f}")
    print(f"{'total':24s} {lane.sum():10.2f} {wave.sum():14.2f}")


if __name__ == "__main__":
    main()
