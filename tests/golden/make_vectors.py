"""Writes the committed golden vectors (tests/golden/vectors_*.npz): small
seeded bursts of every config shape plus an edge-corpus burst, with the
oracle's outputs (dp_pkt_out_t records and the rewritten buffer).

    python tests/golden/make_vectors.py

The tables are rebuilt from the same seeded generators when the vectors are
checked; `tables_digest` pins that the generators still produce the same
tables.  Test infrastructure (imports the oracle)."""
import ctypes
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.dirname(os.path.dirname(HERE))]

import numpy as np  # noqa: E402

from dataplane_amd import _abi as A  # noqa: E402
from dataplane_amd.workload import Workload  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

VECTORS = {  # name -> (config, packets, seed, table knobs)
    "c1": (1, 512, 11, dict(n_routes_v4=2000)),
    "c2": (2, 512, 12, dict(n_routes_v4=4000, n_acl=300, n_nat=32, tcp_percent=30)),
    "c3": (3, 256, 13, dict(n_routes_v4=4000, n_acl=300, n_nat=32, tcp_percent=30)),
    "c4": (4, 512, 14, dict(n_routes_v4=4000, n_acl=300, n_nat=32, tcp_percent=30)),
    "c5": (5, 512, 15, dict(n_routes_v4=4000, n_routes_v6=2000, n_acl=300, n_nat=32,
                            tcp_percent=30)),
}


def tables_digest(tp) -> str:
    """sha256 over every descriptor array's bytes."""
    d = tp.contents
    h = hashlib.sha256()
    for name, _ in A.TablesDesc._fields_:
        if name.startswith("n_") or name in ("abi_version", "pad0", "genid", "masq_config_tag",
                                              "masq_randomize", "pad1", "masq_seed"):
            continue
        n = getattr(d, "n_" + name)
        if n:
            arr = getattr(d, name)
            h.update(name.encode() + ctypes.string_at(arr, n * ctypes.sizeof(arr._type_)))
    return h.hexdigest()


def workload(name):
    cfg, n, seed, kw = VECTORS[name]
    return Workload(cfg, n, seed=seed, **kw)


def edge_burst():
    sys.path.insert(0, os.path.dirname(HERE))
    from edgecase import edge_frames, edge_tables, pack_burst
    t = edge_tables()
    tp = t.build()
    buf, inp = pack_burst(edge_frames(1500, 4242))
    return t, tp, buf, inp


def main():
    for name in VECTORS:
        w = workload(name)
        b = w.fresh_buf()
        out = Oracle(w.tables).process(b, w.inp)
        np.savez_compressed(os.path.join(HERE, f"vectors_{name}.npz"), buf_in=w.buf, inp=w.inp,
                            out=out, buf_out=b, tables_digest=np.array(tables_digest(w.tables)))
        print(name, w.n, "packets")
    t, tp, buf, inp = edge_burst()
    b = buf.copy()
    out = Oracle(tp).process(b, inp)
    np.savez_compressed(os.path.join(HERE, "vectors_edge.npz"), buf_in=buf, inp=inp, out=out,
                        buf_out=b, tables_digest=np.array(tables_digest(tp)))
    print("edge", len(inp), "packets")


if __name__ == "__main__":
    main()
