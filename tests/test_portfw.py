"""Port forwarding on the oracle (CPU): the reference's PortForwarder tests
(nat/src/portfw/test.rs) as scenarios (tests/golden/pfkat.py), and the rule
table's update semantics (PortFwTable::update, objects.rs:284-300)."""
import pytest

from golden import pfkat


@pytest.mark.parametrize("s", pfkat.scenarios(), ids=lambda s: s.name)
def test_oracle_portfw_kat(s):
    errs = pfkat.run_scenario(s, pfkat.OracleRunner())
    assert not errs, "\n".join(errs)


def test_oracle_portfw_rule_lineage():
    """An entry that matches one of the previous generation keeps its id (its
    Weak upgrades); a changed rule is a new entry; an overlapping rule of the
    same key and prefix is refused (test_port_forwarding_table_updates /
    _removals / test_port_forwarder_rule_insertion, objects.rs:537-620,
    portforwarder.rs:117-151)."""
    from oracle.pyoracle import Oracle
    keep = []

    def tabs(rules, prev=None):
        b = pfkat.world(rules)()
        keep.append(b)
        return Oracle(b.build(), prev=prev)
    r1 = pfkat.tcp_rule()
    o1 = tabs([r1])
    assert o1.rule_alive(1) and not o1.rule_alive(2)
    o2 = tabs([dict(r1, init_timeout_s=13, estab_timeout_s=99)], o1)   # same entry, new timers
    assert o2.rule_alive(1)
    o3 = tabs([dict(r1, int_prefix="192.168.9.1/32")], o2)              # another entry
    assert not o3.rule_alive(1) and o3.rule_alive(2)
    # same key and prefix, overlapping ports: the later rule is added first
    # (the set is applied last to first), the earlier one is refused
    o4 = tabs([pfkat.tcp_rule(ext_ports=(3000, 3022), int_ports=(1000, 1022)),
               pfkat.tcp_rule(ext_ports=(3022, 3022), int_ports=(1022, 1022))], o3)
    assert o4.rule_alive(3) and not o4.rule_alive(4)
    # a removal kills the Weak even if the same rule comes back later
    o5 = tabs([], o4)
    o6 = tabs([pfkat.tcp_rule(ext_ports=(3022, 3022), int_ports=(1022, 1022))], o5)
    assert not o6.rule_alive(3) and o6.rule_alive(4)


def test_oracle_portfw_random_bursts():
    """The seeded port-forwarding bursts (tests/pfgen.py) through the oracle:
    every kind of outcome occurs, and the flow table holds pairs."""
    import pfgen
    from dataplane_amd import _abi as A
    seen = {}

    def on_burst(k, res, buf, infos, look):
        for d in res["done"]:
            seen[A.DONE_NAMES[d]] = seen.get(A.DONE_NAMES[d], 0) + 1
    r = pfkat.OracleRunner()
    pfgen.run(r, seed=3, n_conn=300, on_burst=on_burst)
    assert seen.get("Delivered", 0) > 500 and seen.get("NatNotPortForwarded", 0) > 10
    ln, act = r.count()
    assert ln > 200 and ln % 1 == 0 and act <= ln
