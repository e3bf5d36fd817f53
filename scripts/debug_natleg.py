"""Debug aid: one NAT-leg launch (dataplane_amd/natwork.py) with the
DP_DEBUG_NAT library: how many NAT records the parallel pass processed."""
import ctypes as C
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from dataplane_amd import _abi as A, natwork as W, GpuPathNf
from dataplane_amd.flows import FlowTable

n, share = int(sys.argv[1]), float(sys.argv[2])
lib = A.gpu_lib()
lib.dpf_debug_nat_records.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
lib.dpf_debug_nat_record_bytes.restype = C.c_uint32
Wd = lib.dpf_debug_nat_record_bytes() // 4
nf = GpuPathNf(0)
nf.publish(W.tables().build())
ft = FlowTable(0, 1 << 23)
nf.attach_flows(ft)
buf, inp, npf = W.burst(n, share, 0)
res = nf.process_arrays(buf, inp)
cnt = np.zeros(8, np.uint32)
raw = np.zeros(n * Wd, np.uint32)
lib.dpf_debug_nat_records(nf.ctx, cnt.ctypes.data, raw.ctypes.data, n, None, None)
raw = raw.reshape(n, Wd)[:cnt[0]]
print("counters", cnt.tolist(), "pf packets", npf, "flows", ft.count())
pc = raw[:, 47]
print("processed counts:", {int(c): int((pc == c).sum()) for c in np.unique(pc)})
print("done:", {A.DONE_NAMES[d]: int(c) for d, c in zip(*np.unique(res["done"], return_counts=True))})
