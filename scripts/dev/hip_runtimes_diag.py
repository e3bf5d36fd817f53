"""Diagnostic (GPU box): the round-5 "ACL results left unwritten" anomaly.

Each leg runs in its own process: the ACL classifier over host memory
(dp_acl_classify, and dp_acl_classify_match per family) on the C2 / C5
workloads with BASELINE's 10k rules, six rounds, every result compared with
the oracle.  Legs:
  torch_first/async        torch's HIP runtime first (one runtime), the
                           round-5 copies (hipMemcpyAsync to / from pageable
                           memory)
  lib_loaded_first/async   libdpgpu.so mapped first, torch's runtime mapped
                           after it and initialised first: two HIP runtimes
                           (the dp_ctx_create guard bypassed), round-5 copies
  lib_loaded_first/pinned  the same, the pinned, stream-ordered copies
  lib_inits_first          two runtimes, the library's initialised first
  default                  the product as shipped (one runtime, pinned)
Prints per leg: HIP runtimes mapped, calls, calls with wrong results."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def leg(order: str, copies: int) -> dict:
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    if order == "torch_first":
        import torch
        torch.cuda.init()
    from dataplane_amd import GpuPathNf, _abi as A
    lib = A.gpu_lib()
    if order == "lib_loaded_first":
        # the library mapped first (its runtime not yet initialised), then
        # torch maps its own and initialises it first: the round-5 test
        # sessions whose collection loaded libdpgpu.so before the fixture
        # initialised torch
        import torch
        torch.cuda.init()
        x = torch.ones(1 << 20, device="cuda")
        torch.cuda.synchronize()
    nf0 = GpuPathNf(0)
    if order == "lib_inits_first":
        # the library's runtime initialises the device first, then torch's
        import torch
        try:
            torch.cuda.init()
        except RuntimeError as e:
            nf0.close()
            return {"order": order, "hip_runtimes_mapped": int(lib.dpd_debug_hip_runtimes()),
                    "torch": str(e)}
    lib.dpd_debug_classify_copies(copies)
    from dataplane_amd.workload import Workload
    from oracle.pyoracle import Oracle
    import test_acl_classify as T
    calls = bad = 0
    for cfg in (5, 2, 5, 5, 2, 5):
        w = Workload(cfg, 20000, seed=90 + cfg, n_routes_v4=4000, n_routes_v6=2000, n_acl=10000, n_nat=16)
        o = Oracle(w.tables)
        res = o.process(w.fresh_buf(), w.inp)
        _, keys = T.keys_of(w, res, res)
        keys = np.concatenate([keys, T.perturb(keys, 10 + cfg)])
        keys = keys[np.isin(keys["family"], [4, 6])]
        want = o.acl_classify(keys)
        o.close()
        nf = GpuPathNf(0)
        nf.publish(w.tables)
        for _ in range(int(os.environ.get("DIAG_REPS", "8"))):
            got = nf.acl_classify(keys)
            calls += 1
            bad += int(not all(np.array_equal(got[f], want[f]) for f in ("rule", "action", "scope", "acl")))
            for fam in (4, 6):
                sel, buf, size, st = T.match_keys(keys, fam, 48)
                m = keys["family"] == fam
                got = nf.acl_classify_match(buf, size, st)
                calls += 1
                bad += int(not all(np.array_equal(got[f], want[f][m]) for f in ("rule", "action", "scope", "acl")))
        nf.close()
    nf0.close()
    return {"order": order, "copies": ["pinned", "async_pageable"][copies],
            "hip_runtimes_mapped": int(lib.dpd_debug_hip_runtimes()), "calls": calls, "wrong_calls": bad}


if __name__ == "__main__":
    if len(sys.argv) > 1:
        order, copies = sys.argv[1], int(sys.argv[2])
        print(json.dumps(leg(order, copies)), flush=True)
        sys.exit(0)
    two = {"DPGPU_NO_RUNTIME_PRELOAD": "1", "DPGPU_ALLOW_TWO_HIP_RUNTIMES": "1"}
    legs = [("torch_first", 1, {}), ("lib_loaded_first", 1, two), ("lib_loaded_first", 0, two),
            ("lib_inits_first", 1, two), ("default", 0, {})]
    for order, copies, env in legs:
        r = subprocess.run([sys.executable, __file__, order, str(copies)], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=600)
        line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
        print(line or json.dumps({"order": order, "copies": copies, "rc": r.returncode,
                                  "stderr": r.stderr[-600:]}), flush=True)
