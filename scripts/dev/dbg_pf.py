"""Diagnostic: one port-forwarding scenario on the GPU and the oracle, the
packet's flow and its related flow after every step."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "tests"), os.path.join(os.path.dirname(__file__), "..", "..")]
import torch
torch.cuda.init()
from golden import pfkat
from dataplane_amd import _abi as A
name = sys.argv[1] if len(sys.argv) > 1 else "tcp_close_server"
s = [x for x in pfkat.scenarios() if x.name == name][0]
for mk in (pfkat.OracleRunner, pfkat.GpuRunner):
    r = mk()
    def on_step(i, res, buf, info):
        o = res[0]
        rel = None
        if info is not None and info["related"] != A.FLOW_NONE:
            rel = r.get([info["related"]])[0]
        f = lambda x: None if x is None else (int(x["status"]), int(x["pf"]), int(x["pf_status"]), int(x["pf_rule"]), int(x["expires_at"]) // 10**9)
        print(mk.__name__, i, A.DONE_NAMES[o["done"]] if o["done"] < 34 else o["done"], "flow", f(info), "rel", f(rel), "count", r.count())
    print(pfkat.run_scenario(s, r, on_step))
