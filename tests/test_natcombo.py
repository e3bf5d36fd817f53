"""The NAT stages composed on the oracle (CPU): the reference's NAT pipeline
tests (nat/src/test.rs) as scenarios (tests/golden/natcombo.py) -- static NAT
with masquerade, static NAT with port forwarding, both with ICMP errors, and
a masquerade expose overlapping a port-forwarding expose on one public
address."""
import pytest

from golden import masqkat, natcombo


@pytest.mark.parametrize("s", natcombo.scenarios(), ids=lambda s: s.name)
def test_oracle_natcombo_kat(s):
    errs = masqkat.run_scenario(s, masqkat.OracleRunner())
    assert not errs, "\n".join(errs)
