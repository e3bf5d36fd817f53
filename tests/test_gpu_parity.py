"""GPU parity: the HIP path (through the C ABI) against the oracle on the
same seeded bursts.  Bit-exact on metadata and serialized bytes."""
import numpy as np
import pytest

from dataplane_amd import GpuPathNf, _abi as A
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle

from helpers import compare, hist

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nf():
    n = GpuPathNf(0)
    yield n
    n.close()


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_gpu_matches_oracle(nf, cfg):
    w = Workload(cfg, 20000, seed=200 + cfg, n_routes_v4=20000, n_routes_v6=8000, n_acl=1000,
                 n_nat=64, tcp_percent=25)
    nf.publish(w.tables)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp, A.PKT_OUT)
    stats = np.zeros(A.DONE_COUNT, dtype=np.uint64)
    o_dut = nf.process_arrays(b_dut, w.inp, stats)
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg}")
    h = hist(o_ref)
    assert int(stats.sum()) == w.n
    assert int(stats[A.DONE["Delivered"]]) == h.get("Delivered", 0)
