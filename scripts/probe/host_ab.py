"""A/B of the staged host path's byte moves (dp_process_burst, DP_HOST_COPY):
streaming 16-byte stores into pinned staging + 16-byte write-back moves
against plain memcpy (DPGPU_HOST_PLAIN), alternating in one process on the
C2 burst; DPGPU_HOST_TRACE prints each burst's host phases to stderr."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from dataplane_amd import GpuPathNf, _abi as A  # noqa: E402
from dataplane_amd.workload import Workload  # noqa: E402


def main():
    torch.cuda.init()
    w = Workload(2, 2_000_000, seed=1, layout="dpdk")
    nf = GpuPathNf(0)
    nf.publish(w.tables)
    nf.set_host_path(A.HOST_COPY)

    def pinned(nbytes):
        return torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy()
    pnp = pinned(w.buf.nbytes)
    pin_in = pinned(w.inp.nbytes).view(A.PKT_IN)
    pin_in[:] = w.inp
    pin_out = pinned(w.n * A.PKT_OUT.itemsize).view(A.PKT_OUT)
    ref = None
    res = {"stream": [], "plain": []}
    for r in range(14):
        mode = "plain" if r % 2 else "stream"
        if mode == "plain":
            os.environ["DPGPU_HOST_PLAIN"] = "1"
        else:
            os.environ.pop("DPGPU_HOST_PLAIN", None)
        pnp[:] = w.buf
        t0 = time.perf_counter()
        nf.process_arrays(pnp, pin_in, out=pin_out, with_meta=False)
        dt = time.perf_counter() - t0
        if ref is None:
            ref = (pnp.copy(), pin_out.copy())
        else:
            assert np.array_equal(ref[0], pnp) and np.array_equal(ref[1], pin_out), mode
        if r >= 2:
            res[mode].append(dt)
        print(f"{mode:7s} {dt * 1e3:7.2f} ms", flush=True)
    for k, v in res.items():
        m = sorted(v)[len(v) // 2]
        print(f"{k:7s} median {m * 1e3:.2f} ms  {w.n / m / 1e6:.1f} Mpps")
    nf.close()


if __name__ == "__main__":
    main()
