"""Debug aid: run one masqgen seed on the oracle and the GPU and print where
they first differ (flows by key before a burst, then the burst's packets)."""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import numpy as np
import masqgen
from golden import masqkat as M
from dataplane_amd import _abi as A
from helpers import common_fields

seed, n = int(sys.argv[1]), int(sys.argv[2])
INFO = ("status", "flags", "dst_vni", "genid", "expires_at", "masq", "masq_alloc", "pf_status", "pf_port", "pf_ip")
got = {}
for name, mk in (("oracle", M.OracleRunner), ("gpu", M.GpuRunner)):
    r = mk(slots=1 << 15) if name == "gpu" else mk()
    pre, post = [], []
    masqgen.run(r, seed, n, None,
                lambda k, res, buf, infos, look, rel, pkts: post.append((res.copy(), infos.copy(), look.copy(), rel.copy(), pkts)),
                lambda k, look: pre.append((look.copy(), r.get(look["related"]).copy())))
    got[name] = (pre, post)
(po, so), (pg, sg) = got["oracle"], got["gpu"]
def show(tag, x):
    return f"{tag}: ref={'-' if x['ref'] == A.FLOW_NONE else 'y'} " + " ".join(f"{k}={x[k]}" for k in INFO)
for k in range(len(so)):
    (lo, ro), (lg, rg) = po[k], pg[k]
    for i in range(len(lo)):
        for what, a, b in (("fwd", lo[i], lg[i]), ("rev", ro[i], rg[i])):
            if any(not np.array_equal(a[f], b[f]) for f in INFO) or ((a["ref"] == A.FLOW_NONE) != (b["ref"] == A.FLOW_NONE)):
                print(f"before burst {k}: conn {i} {what}\n  {show('o', a)}\n  {show('g', b)}")
    res_o, inf_o, _, _, pk = so[k]
    res_g, inf_g, _, _, _ = sg[k]
    a, b = common_fields(res_o, res_g)
    bad = np.nonzero(a != b)[0]
    for j in bad[:5]:
        f = M.out_fields(pk[j].frame)
        print(f"burst {k} pkt {j} vni {pk[j].vni} {f}\n  o {a[j]}\n  g {b[j]}\n  {show('o-flow', inf_o[j])}\n  {show('g-flow', inf_g[j])}")
        # the same connection's other packets of the burst
        for q in range(len(pk)):
            fq = M.out_fields(pk[q].frame)
            if {fq['src'], fq['dst']} == {f['src'], f['dst']} and q != j:
                print(f"    pkt {q} {fq} -> o {A.DONE_NAMES[res_o[q]['done']]} g {A.DONE_NAMES[res_g[q]['done']]}")
    if len(bad):
        break
