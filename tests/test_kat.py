"""CPU: the reference's known-answer tests (tests/golden/kat.py) through the
oracle and through the kernel's per-packet code compiled for the host."""
import pytest

from dataplane_amd import _abi as A
from oracle.pyoracle import Oracle
import pyemu

from golden.kat import all_cases, run_case

CASES = all_cases()


def oracle_process(tp, buf, inp):
    return Oracle(tp).process(buf, inp)


def emu_process(tp, buf, inp):
    return pyemu.process(tp, buf, inp)


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_kat_oracle(case):
    errs = run_case(case, oracle_process)
    assert not errs, "\n".join(errs)


@pytest.mark.parametrize("case", CASES, ids=[c.name for c in CASES])
def test_kat_emu(case):
    errs = run_case(case, emu_process)
    assert not errs, "\n".join(errs)
