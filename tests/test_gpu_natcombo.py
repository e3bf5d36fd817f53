"""GPU: the NAT stages composed (static NAT, port forwarding, masquerade and
their ICMP errors) through the C ABI against the oracle -- the reference's NAT
pipeline tests (nat/src/test.rs, as tests/golden/natcombo.py scenarios), every
step compared bit-exactly: records, delivered bytes, the packet's flow."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from golden import masqkat, natcombo
from helpers import common_fields
from test_gpu_masquerade import same_info

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def torch_first():
    import torch
    torch.cuda.init()


@pytest.mark.parametrize("s", natcombo.scenarios(), ids=lambda s: s.name)
def test_gpu_natcombo_kat(s):
    steps_o, steps_g = [], []
    errs = masqkat.run_scenario(s, masqkat.OracleRunner(),
                                lambda i, res, buf, info: steps_o.append((res.copy(), buf.copy(), info)))
    assert not errs, errs
    g = masqkat.GpuRunner()
    try:
        errs = masqkat.run_scenario(s, g, lambda i, res, buf, info: steps_g.append(
            (res.copy(), buf.copy(), info)))
    finally:
        g.close()
    assert not errs, "\n".join(errs)
    assert len(steps_o) == len(steps_g)
    for i, ((ro, bo, io), (rg, bg, ig)) in enumerate(zip(steps_o, steps_g)):
        a, b = common_fields(ro, rg)
        assert np.array_equal(a, b), f"step {i}: records {a} != {b}"
        o = ro[0]
        if o["done"] == A.DONE["Delivered"]:
            assert bo[o["off"]:o["off"] + o["len"]].tobytes() == bg[o["off"]:o["off"] + o["len"]].tobytes(), \
                f"step {i}: frame"
        assert (io is None) == (ig is None), f"step {i}: flow attached"
        if io is not None:
            same_info(io, ig, f"step {i}")
