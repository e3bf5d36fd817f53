"""The C-ABI library loads and exports every symbol include/dpgpu.h declares;
the ctypes mirror matches the C struct layouts.  No GPU compute here."""
import ctypes as C
import os
import re

from dataplane_amd import _abi as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "dpgpu.h")).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(dp_\w+)\(", src, flags=re.M)))


def test_header_symbols_match_list():
    assert declared_symbols() == sorted(A.GPU_SYMBOLS)


def test_library_exports_every_symbol():
    lib = A.gpu_lib()
    for s in A.GPU_SYMBOLS:
        assert hasattr(lib, s), s
    assert lib.dp_abi_version() == A.ABI_VERSION


def test_struct_layouts_match_c():
    lib = A.work_lib()
    for name, st in A.STRUCTS.items():
        assert C.sizeof(st) == lib.dpw_sizeof(name.encode()), name
    assert lib.dpw_sizeof(b"dp_pkt_in_t") == A.PKT_IN.itemsize
    assert lib.dpw_sizeof(b"dp_pkt_out_t") == A.PKT_OUT.itemsize
    assert lib.dpw_sizeof(b"dp_pkt_meta_t") == A.PKT_META.itemsize
    assert C.sizeof(A.MbufLayout) == lib.dpw_sizeof(b"dp_mbuf_layout_t")
    for name, dt in A.NP_STRUCTS.items():
        assert dt.itemsize == lib.dpw_sizeof(name.encode()), name


def test_ctx_create_without_gpu_fails_loudly():
    """No silent CPU fallback: without a device the context cannot be created."""
    import torch
    if torch.cuda.is_available():
        return
    lib = A.gpu_lib()
    h = C.c_void_p()
    assert lib.dp_ctx_create(0, C.byref(h)) == -19  # DP_ENODEV


_RUNTIME_PROBE = '''
import ctypes as C, os, sys
sys.path.insert(0, {root!r})
{pre}
from dataplane_amd import _abi as A
lib = A.gpu_lib()
import torch
h = C.c_void_p()
print(lib.dpd_debug_hip_runtimes(), lib.dp_ctx_create(0, C.byref(h)) if not torch.cuda.is_available() else 0)
'''


def _runtime_probe(pre: str, env: dict):
    import subprocess
    import sys
    r = subprocess.run([sys.executable, "-c", _RUNTIME_PROBE.format(root=ROOT, pre=pre)],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return [int(x) for x in r.stdout.split()]


def test_one_hip_runtime_per_process():
    """libdpgpu.so loaded before PyTorch: the Python mirror maps PyTorch's
    HIP runtime first, so one runtime serves both; either
    import order gives one."""
    n, rc = _runtime_probe("", {})
    assert n == 1
    n, rc = _runtime_probe("import torch", {})
    assert n == 1


def test_two_hip_runtimes_refused():
    """Without that (the preload disabled, the library first), PyTorch maps a
    second runtime beside the library's; dp_ctx_create refuses the process
    (DP_ENOTSUP) before touching any device."""
    n, rc = _runtime_probe("", {"DPGPU_NO_RUNTIME_PRELOAD": "1"})
    assert n == 2
    import torch
    if not torch.cuda.is_available():
        assert rc == -95  # DP_ENOTSUP
