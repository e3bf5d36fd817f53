"""The already-serialized contract of the boundary: the
driver rebuilds each delivered packet with Packet::new from the output frame
and transmits it through Packet::serialize (dataplane/src/drivers/kernel/
worker.rs:577).  That must send the output frame unchanged: parse +
update_checksums + deparse of every delivered frame is the identity.  Checked
on the committed golden outputs (oracle outputs; the GPU matches them
byte for byte in tests/test_gpu_parity.py)."""
import os

import numpy as np
import pytest

from dataplane_amd import _abi as A
from golden.make_vectors import VECTORS
from oracle.pyoracle import reserialize

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", list(VECTORS) + ["edge"])
def test_delivered_frames_reserialize_unchanged(name):
    z = np.load(os.path.join(HERE, f"vectors_{name}.npz"))
    out, buf = z["out"], z["buf_out"]
    n = 0
    for r in out[out["done"] == A.DONE["Delivered"]]:
        frame = bytes(buf[r["off"]:r["off"] + r["len"]])
        again = reserialize(frame)
        assert again == frame, f"{name}: frame at {int(r['off'])} changes when re-sent"
        n += 1
    assert n > 0
