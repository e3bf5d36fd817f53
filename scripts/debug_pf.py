"""Debug aid: pfgen seed on the GPU (parallel NAT pass) against the oracle;
the first burst that differs, with the NAT records and connection lists of
the differing packets."""
import ctypes as C
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import pfgen
from golden import pfkat
from dataplane_amd import _abi as A
from helpers import common_fields

seed, n = int(sys.argv[1]), int(sys.argv[2])
lib = A.gpu_lib()
lib.dpf_debug_nat_records.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
lib.dpf_debug_nat_record_bytes.restype = C.c_uint32
W = lib.dpf_debug_nat_record_bytes() // 4
got = {}
for name, mk in (("oracle", pfkat.OracleRunner), ("gpu", pfkat.GpuRunner)):
    r = mk(slots=1 << 14) if name == "gpu" else mk()
    steps = []
    def cb(k, res, buf, infos, look):
        extra = None
        if name == "gpu":
            cnt = np.zeros(8, np.uint32)
            m = len(res)
            raw = np.zeros(m * W, np.uint32)
            nxt = np.zeros(m, np.uint64)
            heads = np.zeros(m, np.uint64)
            lib.dpf_debug_nat_records(r.nf.ctx, cnt.ctypes.data, raw.ctypes.data, m, nxt.ctypes.data,
                                      heads.ctypes.data)
            extra = (cnt.copy(), raw.reshape(m, W).copy(), nxt.copy(), heads[:cnt[4]].copy())
        steps.append((res.copy(), infos.copy(), extra))
    pfgen.run(r, seed, n, None, cb)
    got[name] = steps
for k, ((ro, io, _), (rg, ig, ex)) in enumerate(zip(got["oracle"], got["gpu"])):
    a, b = common_fields(ro, rg)
    bad = np.nonzero(a != b)[0]
    cnt, raw, nxt, heads = ex
    print(f"burst {k}: counters {cnt.tolist()}, {len(bad)} differ")
    if not len(bad):
        continue
    nrec = int(cnt[0])
    rec_of = {int(raw[r, 0]): r for r in range(nrec)}
    # the lists as the resolve kernel walked them (sorted in place)
    seen = {}
    for e, hd in enumerate(heads):
        r = int(hd & 0xffffffff)
        chain = []
        while r != 0xffffffff and len(chain) < 10000:
            chain.append(r)
            r = int(nxt[r] & 0xffffffff)
        for x in chain:
            seen.setdefault(x, []).append(e)
    indeg = {}
    for r in range(nrec):
        t = int(nxt[r] & 0xffffffff)
        if t != 0xffffffff:
            indeg[t] = indeg.get(t, 0) + 1
    print("records with 2+ predecessors:", sum(1 for v in indeg.values() if v > 1),
          "chains:", sum(1 for r in range(nrec) if raw[r, 1] & 1 and r not in indeg), "groups:", int(cnt[4]))
    print("group heads:", len(heads), "distinct:", len(set(int(x) for x in heads)))
    pc = raw[:nrec, 47]
    print("processed counts:", {int(c): int((pc == c).sum()) for c in np.unique(pc)})
    for i in bad[:6]:
        r = rec_of.get(int(i))
        if r is None:
            print(" pkt", i, "no record"); continue
        w = raw[r]
        print(f" pkt {i} rec {r}: bits {w[1]:#x} slot {w[2]} state {w[3]:#x} status0 {w[4]} fflags0 {w[5]:#x} "
              f"src_vni {w[6]} verdict {w[37]} lane {w[46]} times {w[47]} next {nxt[r] >> 32}/{nxt[r] & 0xffffffff:#x}")
    break
