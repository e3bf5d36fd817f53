"""The randomized masquerade allocator (MasqueradeConfig::set_randomize(true),
the reference's default, nat/src/masquerade/allocator_writer.rs:58, set by
mgmt, mgmt/src/processor/proc.rs:541): each address's 256 port blocks come in
a shuffled order (PortAllocator::new, nat/src/masquerade/apalloc/
port_alloc.rs:105-113).  dpgpu.h specifies the shuffle as a function of
masq_seed and the address; `block_order` below restates that specification a
third time (beside the oracle's and the device's) and pins the oracle to it:

- CPU: the ports handed to a run of first packets come block by block in the
  permuted order (position by position from current_alloc_index, the IANA
  well-known blocks skipped), ports in order within a block; another seed
  gives another order; randomize = false gives blocks 4, 5, 6, ...
- GPU: the same burst, and the seeded masquerade bursts of tests/masqgen.py
  (exhaustion, repeats, replies, closes, republish, narrowed config) for two
  seeds, GPU == oracle (tests/test_gpu_masquerade.py's comparison)."""
import numpy as np
import pytest

from dataplane_amd import _abi as A
from dataplane_amd import natwork as W
from golden.masqkat import OracleRunner

M64 = (1 << 64) - 1


def splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def block_order(seed: int, addr: int) -> list:
    """dpgpu.h's permutation: perm[i] = the random_index of block i."""
    x = seed
    for k in (3, 2, 1, 0):
        x = splitmix64(x ^ ((addr >> (32 * k)) & 0xFFFFFFFF))
    p = list(range(256))
    for i in range(255, 0, -1):
        x = splitmix64(x)
        j = x % (i + 1)
        p[i], p[j] = p[j], p[i]
    return p


def expected_ports(perm, n):
    """The first n ports of a fresh address (UDP: the well-known blocks
    excluded, no claims): block positions from 0, each block's ports in order."""
    out = []
    for i in range(256):
        if perm[i] < 4:
            continue
        out.extend(range(perm[i] * 256, perm[i] * 256 + 256))
        if len(out) >= n:
            break
    return out[:n]


def first_ports(run_burst, seed):
    t = W.masq_world()
    if seed is not None:
        t.masq_randomize, t.masq_seed = True, seed
    c = W.MasqConns(3000)
    buf, inp = c.first()
    out = run_burst(t, buf, inp)
    assert np.all(out["done"] == A.DONE["Delivered"])
    assert c.learn(buf, out) == 3000
    return c.pub.copy(), c.pport.astype(np.int64)


def oracle_burst(t, buf, inp):
    r = OracleRunner()
    r.publish(t)
    r.set_clock(10 ** 12)
    return r.burst(buf, inp)


@pytest.mark.parametrize("seed", [None, 1, 0xDEADBEEF])
def test_oracle_ports_follow_the_block_order(seed):
    pub, ports = first_ports(oracle_burst, seed)
    base = 203 << 24 | 0 << 16 | 113 << 8
    assert np.all(pub == base)  # one address holds them all
    perm = block_order(seed, base) if seed is not None else list(range(256))
    assert ports.tolist() == expected_ports(perm, 3000)
    if seed is not None:
        assert perm != list(range(256))


def test_block_order_is_a_permutation_per_seed_and_address():
    a = block_order(1, 0xCB007100)
    assert sorted(a) == list(range(256))
    assert a != block_order(2, 0xCB007100) and a != block_order(1, 0xCB007101)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [7, 0x5EED])
def test_gpu_randomized_allocator(seed):
    import torch
    torch.cuda.init()
    from golden.masqkat import GpuRunner

    def gpu_burst(t, buf, inp):
        r = GpuRunner(slots=1 << 14)
        try:
            r.publish(t)
            r.set_clock(10 ** 12)
            return r.burst(buf, inp)
        finally:
            r.close()
    po, qo = first_ports(oracle_burst, seed)
    pg, qg = first_ports(gpu_burst, seed)
    assert np.array_equal(po, pg) and np.array_equal(qo, qg)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [7, 0x5EED])
def test_gpu_randomized_random_bursts(seed):
    import torch
    torch.cuda.init()
    import masqgen
    from golden.masqkat import GpuRunner
    from test_gpu_masquerade import same_info
    from helpers import common_fields
    got = {}
    for name, mk in (("oracle", OracleRunner), ("gpu", GpuRunner)):
        r = mk(slots=1 << 15) if name == "gpu" else mk()
        steps = []
        try:
            masqgen.run(r, 4, 3000, None, lambda k, res, buf, infos, look, rel, pkts: steps.append(
                (res.copy(), buf.copy(), infos.copy(), look.copy(), rel.copy(), r.count())), randomize_seed=seed)
        finally:
            if name == "gpu":
                r.close()
        got[name] = steps
    for k, (o, g) in enumerate(zip(got["oracle"], got["gpu"])):
        (ro, bo, io, lo, xo, co), (rg, bg, ig, lg, xg, cg) = o, g
        a, b = common_fields(ro, rg)
        assert np.array_equal(a, b), f"burst {k}: records"
        d = ro["done"] == A.DONE["Delivered"]
        for i in np.nonzero(d)[0]:
            s0, n0 = int(ro[i]["off"]), int(ro[i]["len"])
            assert np.array_equal(bo[s0:s0 + n0], bg[s0:s0 + n0]), f"burst {k} packet {i}: frame"
        same_info(io, ig, f"burst {k}: packets'")
        same_info(lo, lg, f"burst {k}: flows by key:")
        same_info(xo, xg, f"burst {k}: related flows:")
        assert co == cg
