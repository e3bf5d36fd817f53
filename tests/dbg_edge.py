"""Debug helper: show one packet of the edge corpus through oracle and emu.
    python tests/dbg_edge.py SEED INDEX [N]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.join(HERE, "emu"), os.path.dirname(HERE)]

from dataplane_amd import _abi as A  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402
import pyemu  # noqa: E402
from edgecase import edge_frames, edge_tables, pack_burst  # noqa: E402


def main():
    seed, idx = int(sys.argv[1]), int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 4000
    t = edge_tables()
    tp = t.build()
    frames = edge_frames(n, seed)
    fr = frames[idx]
    buf, inp = pack_burst([fr])
    b1, b2 = buf.copy(), buf.copy()
    o1 = Oracle(tp).process(b1, inp, A.PKT_OUT)
    o2 = pyemu.process(tp, b2, inp, A.PKT_OUT)
    print("in:", inp[0], "frame:", fr[0].hex())
    for name, o, b in (("ref", o1, b1), ("emu", o2, b2)):
        r = o[0]
        print(name, A.DONE_NAMES[r["done"]] if r["done"] < A.DONE_COUNT else r["done"], r)
        print("   ", bytes(b[r["off"]:r["off"] + r["len"]]).hex())


if __name__ == "__main__":
    main()
