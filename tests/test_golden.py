"""CPU: the committed golden vectors (tests/golden/make_vectors.py) -- the
oracle and the host-compiled kernel body must reproduce them byte for byte."""
import os

import numpy as np
import pytest

from dataplane_amd import _abi as A
from oracle.pyoracle import Oracle
import pyemu

from golden.make_vectors import VECTORS, edge_burst, tables_digest, workload
from helpers import compare

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = list(VECTORS) + ["edge"]


def load(name):
    z = np.load(os.path.join(HERE, f"vectors_{name}.npz"))  # allow_pickle=False
    keep = None
    if name == "edge":
        keep, tp, buf, inp = edge_burst()
    else:
        keep = workload(name)
        tp, buf, inp = keep.tables, keep.buf, keep.inp
    assert str(z["tables_digest"]) == tables_digest(tp), "table generator drifted"
    assert np.array_equal(z["buf_in"], buf) and np.array_equal(z["inp"], inp)
    return keep, tp, z


@pytest.mark.parametrize("name", NAMES)
def test_golden_oracle(name):
    keep, tp, z = load(name)
    b = z["buf_in"].copy()
    out = Oracle(tp).process(b, z["inp"])
    compare(z["out"], z["buf_out"], out, b, z["inp"], f"golden {name} oracle")


@pytest.mark.parametrize("name", NAMES)
def test_golden_emu(name):
    keep, tp, z = load(name)
    b = z["buf_in"].copy()
    out = pyemu.process(tp, b, z["inp"])
    compare(z["out"], z["buf_out"], out, b, z["inp"], f"golden {name} emu")
