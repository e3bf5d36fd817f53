"""CPU: the GPU kernel's per-packet code, compiled for the host (tests/emu),
against the oracle on seeded workloads of every config shape, with the
classifiers built in each form (bit-vector, candidate list, automatic)."""
import pytest

from dataplane_amd import _abi as A
from dataplane_amd.workload import Workload
from oracle.pyoracle import Oracle
import pyemu

from helpers import compare


@pytest.mark.parametrize("form,layout", [("auto", "packed"), ("bv", "packed"), ("list", "packed"),
                                         ("auto", "dpdk")])
@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_emu_matches_oracle(cfg, form, layout, cls_form):
    cls_form(pyemu.lib(), form)
    w = Workload(cfg, 3000, seed=100 + cfg, n_routes_v4=3000, n_routes_v6=1500, n_acl=400,
                 n_nat=48, tcp_percent=25, layout=layout)
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    o_dut = pyemu.process(w.tables, b_dut, w.inp)
    bv, lst = pyemu.classifier_forms()
    if cfg != 1:  # C1 has no overlay tables
        if form == "bv":
            assert lst == 0 and bv > 0
        elif form == "list":
            assert lst > 0
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg} {form}")


@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_emu_dir24_8(cfg):
    """More than 64Ki v4 routes: the 24-bit direct table with DIR-24-8 blocks
    for the /25-/32 routes, on the overlay (pair context) and underlay FIBs."""
    w = Workload(cfg, 20000, seed=400 + cfg, n_routes_v4=120000, n_routes_v6=4000, n_acl=400,
                 n_nat=48, tcp_percent=25, layout="dpdk")
    b_ref, b_dut = w.fresh_buf(), w.fresh_buf()
    o_ref = Oracle(w.tables).process(b_ref, w.inp)
    o_dut = pyemu.process(w.tables, b_dut, w.inp)
    compare(o_ref, b_ref, o_dut, b_dut, w.inp, f"C{cfg} dir24-8")

