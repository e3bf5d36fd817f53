import sys, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from dataplane_amd import GpuPathNf, _abi as A
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle
import test_acl_classify as T
for cfg in (5, 2, 5, 5, 2, 5):
    w = Workload(cfg, 20000, seed=90 + cfg, n_routes_v4=4000, n_routes_v6=2000, n_acl=10000, n_nat=16)
    o = Oracle(w.tables)
    res = o.process(w.fresh_buf(), w.inp)
    _, keys = T.keys_of(w, res, res)
    keys = np.concatenate([keys, T.perturb(keys, 10 + cfg)])
    keys = keys[np.isin(keys["family"], [4, 6])]
    want = o.acl_classify(keys)
    nf = GpuPathNf(0)
    nf.publish(w.tables)
    direct = nf.acl_classify(keys)
    print(cfg, "keys", len(keys), "direct ok", all(np.array_equal(direct[f], want[f]) for f in ("rule","action","scope","acl")), np.unique(direct["acl"]), flush=True)
    for fam in (4, 6):
        sel, buf, size, st = T.match_keys(keys, fam, 48)
        got = nf.acl_classify_match(buf, size, st)
        m = keys["family"] == fam
        print(" fam", fam, len(sel), "match ok", all(np.array_equal(got[f], want[f][m]) for f in ("rule","action","scope","acl")), np.unique(got["acl"]), flush=True)
        got2 = nf.acl_classify(sel)
        print("  direct-sel ok", all(np.array_equal(got2[f], want[f][m]) for f in ("rule","action","scope","acl")), flush=True)
    nf.close()
