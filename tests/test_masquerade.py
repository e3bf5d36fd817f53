"""Masquerade on the oracle (CPU): the reference's Masquerade tests
(nat/src/masquerade/test.rs) as scenarios (tests/golden/masqkat.py)."""
import pytest

from golden import masqkat


@pytest.mark.parametrize("s", masqkat.scenarios(), ids=lambda s: s.name)
def test_oracle_masquerade_kat(s):
    errs = masqkat.run_scenario(s, masqkat.OracleRunner())
    assert not errs, "\n".join(errs)
