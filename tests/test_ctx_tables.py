"""Host logic of the LDS context tables (Image.ctx_bytes, dp_tables.cpp): the
VNI slots, the pair map, the PairRecs and the NhRecs are laid out for a
per-workgroup copy when the image has VPC peerings and they fit
DPD_CTX_MAX (7168 B), 16-byte aligned, in that order; otherwise the kernel
reads them from HBM (dp_kernel.hip DP_CTX)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "emu"))
import pyemu  # noqa: E402

from dataplane_amd.workload import Workload  # noqa: E402

CTX_MAX = 7168


def info(tables):
    lib = pyemu.lib()
    lib.dpemu_image_ctx.argtypes = [C.c_void_p, C.c_void_p]
    o = np.zeros(8, np.uint32)
    assert lib.dpemu_image_ctx(C.cast(tables, C.c_void_p), o.ctypes.data) == 0
    return [int(x) for x in o[:5]]


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_ctx_layout(cfg):
    w = Workload(cfg, 256, seed=1)
    vni, pslots, precs, nh, ctx = info(w.tables)
    a16 = lambda x: (x + 15) & ~15
    total = a16(vni * 96) + a16(pslots * 16) + a16(precs * 128) + a16(nh * 32)
    if precs and total <= CTX_MAX:
        assert ctx == total
    else:
        assert ctx == 0
    # the bench configs: overlay images with peerings fit; C1 (underlay) has none
    assert (ctx > 0) == (cfg != 1)
