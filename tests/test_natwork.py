"""The bench's stateful-NAT workloads (dataplane_amd/natwork.py: the
port-forwarding and masquerade legs of bench.py) at a small size.

CPU: the oracle over each world -- every packet delivered, each opening
packet one translated flow pair (port forwarding: destination 192.168.0.0/16
ports 5000-5999; masquerade: source in the 203.0.113.0/24 pool).
GPU: the C ABI's flows variant (parallel NAT pass for port forwarding, one
lane for masquerade) == the oracle on the same bursts, bit-exact, two
bursts in a row, flow counts included; and a burst sharded over two
contexts sharing one flow table (dp_process_burst_sharded) == the same
shards as consecutive bursts of one context."""
import ipaddress

import numpy as np
import pytest

from dataplane_amd import _abi as A
from dataplane_amd import natwork as W
from helpers import compare
from oracle.pyoracle import Oracle, OracleFlows

N = 20000


def world(kind):
    return (W.masq_tables() if kind == "masq" else W.tables()).build()


@pytest.mark.parametrize("kind", ["pf", "masq"])
def test_oracle_natwork(kind):
    o = Oracle(world(kind))
    ft = OracleFlows()
    buf, inp, npf = W.burst(N, 0.05, 0, kind=kind)
    out, _ = o.process_flows(buf, inp, ft)
    assert np.all(out["done"] == A.DONE["Delivered"])
    assert ft.count() == (2 * npf, 2 * npf)
    pool = ipaddress.ip_network("203.0.113.0/24")
    inner = ipaddress.ip_network("192.168.0.0/16")
    hits = 0
    for i in range(len(inp)):
        f = buf[out[i]["off"]:out[i]["off"] + out[i]["len"]]
        src = ipaddress.ip_address(bytes(f[26:30]))
        dst = ipaddress.ip_address(bytes(f[30:34]))
        hits += (src in pool) if kind == "masq" else (dst in inner)
    assert hits == npf


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pf", "masq"])
def test_gpu_natwork(kind):
    import torch
    torch.cuda.init()
    from dataplane_amd import GpuPathNf
    from dataplane_amd.flows import FlowTable
    tp = world(kind)
    o, oft = Oracle(tp), OracleFlows()
    nf, gft = GpuPathNf(0), FlowTable(0, 1 << 16)
    try:
        nf.publish(tp)
        nf.attach_flows(gft)
        pairs = 0
        for step in range(2):
            buf, inp, npf = W.burst(N, 0.05, step, kind=kind)
            pairs += npf
            ob, gb = buf.copy(), buf.copy()
            oout, _ = o.process_flows(ob, inp, oft)
            gout = nf.process_arrays(gb, inp)
            compare(oout, ob, gout, gb, inp, f"{kind} burst {step}")
            assert gft.count() == oft.count()
            assert gft.count()[0] == 2 * pairs
    finally:
        nf.attach_flows(None)
        gft.close()
        nf.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["pf", "masq"])
def test_gpu_natwork_sharded_shared_table(kind):
    """The reference's workers share one Arc<FlowTable>
    (dataplane/src/packet_processor/mod.rs:68,100-120): shards of a burst
    over two contexts attached to one table run as the workers' bursts in
    shard order -- bit-exact against one context taking the shards as
    consecutive bursts on its own table: outputs, bytes, every flow's
    presence and state, the flow counts, and the masquerade allocations
    (the translated sources)."""
    import torch
    torch.cuda.init()
    from dataplane_amd import GpuPathNf
    from dataplane_amd.flows import FlowTable
    tp = world(kind)
    a, b, ref = GpuPathNf(0), GpuPathNf(0), GpuPathNf(0)
    ft, ft_ref = FlowTable(0, 1 << 16), FlowTable(0, 1 << 16)
    try:
        for nf in (a, b, ref):
            nf.publish(tp)
        a.attach_flows(ft)
        b.attach_flows(ft)
        ref.attach_flows(ft_ref)
        for step in range(2):
            buf, inp, npf = W.burst(N, 0.05, step, kind=kind)
            rb, db = buf.copy(), buf.copy()
            h = len(inp) // 2
            r0 = ref.process_arrays(rb, inp[:h].copy())
            r1 = ref.process_arrays(rb, inp[h:].copy())
            rout = np.concatenate([r0, r1])
            dout = GpuPathNf.process_sharded([a, b], db, inp)
            compare(rout, rb, dout, db, inp, f"{kind} sharded burst {step}")
            assert ft.count() == ft_ref.count()
            assert ft.count()[0] > 0
    finally:
        for nf in (a, b, ref):
            nf.attach_flows(None)
        ft.close()
        ft_ref.close()
        for nf in (a, b, ref):
            nf.close()
