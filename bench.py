# SPDX-License-Identifier: Apache-2.0
"""Benchmark of the MI355X per-burst packet path (BASELINE.json metric).

One step = one pass of the whole path (parse -> Ingress/IP-Forward/flow-filter/
ACL/static NAT/IP-Forward/Egress -> serialize) over one resident burst of
synthetic packets.  Bursts are pre-staged in HBM (one copy per
step, so every step processes pristine packets in place); the timed region
contains only the kernel launches.  Multi-GPU: one process per GPU, each
processing its own shard (packets are independent: weak scaling, no
data-path collective).

Beside `value` (never inside it), rank 0 at N=1 reports legs: the same burst
with meta records, with a flow table attached (flow_table), port forwarding
and masquerade under load (nat_portfw, nat_masquerade: a share of a 2M burst
opening new stateful-NAT connections; nat_mixed: both on one public range),
host-origin bursts (host_inclusive), and the CPU baseline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from dataplane_amd import GpuPathNf, _abi as A  # noqa: E402
from dataplane_amd.shard import reduce_over_ranks, shard_seed, timed_scatter_gather  # noqa: E402
from dataplane_amd.workload import ALGO_BYTES, CONFIG_NAMES, Workload  # noqa: E402

METRIC = "Mpps device-resident (64B IPv4, 1M-route LPM + 10k ACL + NAT) at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def measured_traffic(cfg: int, n: int):
    """HBM traffic per launch from the committed PMC passes (profiles/traffic.json,
    written from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench),
    scaled to this launch's packet count; None when no measurement exists."""
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))[f"C{cfg}"]
    except (OSError, KeyError, ValueError):
        return None, None
    return int(t["bytes_per_pkt"] * n), t["source"]


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def physical_cores(cpus) -> int:
    """Physical cores among the logical CPUs `cpus` (SMT siblings counted
    once), from /sys topology; len(cpus) if unreadable."""
    seen = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            seen.add((open(base + "physical_package_id").read().strip(),
                      open(base + "core_id").read().strip()))
        except OSError:
            return len(cpus)
    return len(seen) or len(cpus)


def cpu_share() -> int:
    """The CPU share this job may load: OMP_NUM_THREADS when the launcher
    sets it (the GPU box sets 16, its per-GPU share -- nproc there shows the
    whole machine), else unlimited."""
    try:
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        return 1 << 30


def cpu_threads() -> int:
    """Host threads for the CPU baseline: one per physical
    core of the affinity mask, within the job's CPU share."""
    return max(1, min(cpu_share(), physical_cores(sorted(os.sched_getaffinity(0)))))


def _time_cpu(run, n: int, budget_s: float, max_reps: int) -> tuple:
    """Repeat run() (which returns its own seconds for n packets) until the
    budget is spent; (Mpps, reps, seconds)."""
    done, t_total, reps = 0, 0.0, 0
    while t_total < budget_s and reps < max_reps:
        t_total += run()
        done += n
        reps += 1
    return done / t_total / 1e6, reps, t_total


def cpu_baseline(w: Workload, sample: int, budget_s: float) -> dict:
    """Two CPU legs on this host, DPDK-sized bursts of 64, bounded samples:
      - "port" (the reported value): the oracle (oracle/), the C++
        restatement of the reference pipeline (linear-scan classifiers,
        binary-trie LPM, like the reference's own reference implementations),
        on cpu_threads() threads and on 1;
      - "compiled": the kernel's per-packet body built for the host
        (tests/emu, -O3) over the same compiled table image (Poptrie LPM,
        candidate-list classifiers), on the same thread counts."""
    from oracle.pyoracle import Oracle  # test-infrastructure checker, timed as the baseline
    sys.path.insert(0, os.path.join(ROOT, "tests", "emu"))
    import pyemu  # test infrastructure (host build of the kernel body)
    threads = cpu_threads()
    o = Oracle(w.tables)

    def oracle_run(m, th):
        inp, out = w.inp[:m].copy(), np.zeros(m, dtype=A.PKT_OUT)

        def run():
            buf = w.fresh_buf()
            t0 = time.perf_counter()
            o.process_parallel(buf, inp, out, threads=th, burst=64)
            return time.perf_counter() - t0
        return run
    n = min(sample, w.n)
    n1 = max(64, n // 8)
    port_n, reps, t_port = _time_cpu(oracle_run(n, threads), n, budget_s, 50)
    port_1, _, _ = _time_cpu(oracle_run(n1, 1), n1, budget_s / 4, 3)
    o.close()

    emu = pyemu.ParallelEmu(w.tables)
    ebuf = pyemu.aligned_copy(w.buf)

    def emu_run(m, th):
        inp, out = w.inp[:m].copy(), np.zeros(m, dtype=A.PKT_OUT)

        def run():
            ebuf[:w.buf.nbytes] = w.buf
            t0 = time.perf_counter()
            emu.run(ebuf, w.buf.nbytes, inp, out, threads=th, burst=64)
            return time.perf_counter() - t0
        return run
    ne = min(w.n, 8 * n)
    emu_n, ereps, t_emu = _time_cpu(emu_run(ne, threads), ne, budget_s / 2, 20)
    emu_1, _, _ = _time_cpu(emu_run(ne // 8, 1), ne // 8, budget_s / 4, 3)
    emu.close()
    aff = sorted(os.sched_getaffinity(0))
    return {"value": round(port_n, 4), "unit": "Mpps", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "value_1_thread": round(port_1, 4),
            "threads_rule": f"one per physical core of the affinity mask ({physical_cores(aff)} "
                            f"physical / {len(aff)} logical CPUs) within the job's CPU share "
                            f"(OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')})",
            "sample": f"{reps} x {n} packets of the same workload, bursts of 64, C++ restatement "
                      f"of the reference pipeline (oracle/), {t_port:.1f} s on {threads} threads; "
                      f"value_1_thread over {n1} packets",
            "compiled": {"value": round(emu_n, 3), "unit": "Mpps", "cores": threads,
                         "value_1_thread": round(emu_1, 3),
                         "what": "the kernel's per-packet body compiled for the host (tests/emu, "
                                 "-O3) over the same table image (Poptrie LPM, candidate lists)",
                         "sample": f"{ereps} x {ne} packets, {t_emu:.1f} s"}}


def flows_leg(nf, w, dev, stream, steps: int) -> dict:
    """The same burst with a flow table attached:
    every other packet belongs to an established flow pair (Active, current
    generation, its destination the packet's own flow-filter verdict), so it
    bypasses the flow-filter tables; the pipeline runs its flows variant
    (FlowLookup on every overlay packet, the flow-aware stages, the fix-up
    and invalidation kernels).  Reported beside `value`, never inside it."""
    from dataplane_amd.flows import FlowTable, burst_request_flows
    n = w.n
    bb = (w.buf.nbytes + 255) & ~255
    pristine = torch.from_numpy(w.buf).to(dev)
    b = torch.empty(bb, dtype=torch.uint8, device=dev)
    dinp = torch.from_numpy(w.inp.view(np.uint8)).to(dev)
    dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
    dmeta = torch.empty(n * A.PKT_META.itemsize, dtype=torch.uint8, device=dev)
    sptr = stream.cuda_stream
    # each packet's flow-filter verdict, from one run without flows
    b[:w.buf.nbytes].copy_(pristine)
    nf.process_device(b.data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n, None, sptr,
                      dev_meta=dmeta.data_ptr())
    torch.cuda.synchronize(dev)
    meta = dmeta.cpu().numpy().view(A.PKT_META)
    # the even packets' request flows (Eth / IPv4 / UDP|TCP frames with a verdict)
    fl = burst_request_flows(w.buf, w.inp, np.arange(0, n, 2), meta["dst_vni"], nf.data.genid)
    slots = 1 << max(12, int(np.ceil(np.log2(max(1, 4 * len(fl))))))
    ft = FlowTable(0, slots)
    ft.set_capacity(len(fl))
    t0 = time.perf_counter()
    _, res = ft.insert(fl)
    t_ins = time.perf_counter() - t0
    nf.attach_flows(ft)
    lib = A.gpu_lib()

    def launches(full):
        # full: the units an image with stateful NAT runs (a port-forwarding
        # rule or a masquerade expose; dpf_debug_flows_full forces them here)
        lib.dpf_debug_flows_full(1 if full else 0)
        try:
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(steps + 2)]
            for k2 in range(steps + 2):
                with torch.cuda.stream(stream):  # on the launch stream: no copy overlaps a launch
                    b[:w.buf.nbytes].copy_(pristine)
                ev[k2][0].record(stream)
                nf.process_device(b.data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n, None, sptr,
                                  dev_meta=dmeta.data_ptr())
                ev[k2][1].record(stream)
            torch.cuda.synchronize(dev)
            lean = lib.dpf_debug_last_lean()
        finally:
            lib.dpf_debug_flows_full(0)
        ms = sorted(a.elapsed_time(c) for a, c in ev[2:])
        return ms[len(ms) // 2], lean

    med_full, lean_f = launches(True)
    med, lean = launches(False)
    refs = dmeta.cpu().numpy().view(A.PKT_META)["flow_ref"]
    hit = int((refs != np.uint64(A.FLOW_NONE)).sum())
    nf.attach_flows(None)
    ln, act = ft.count()
    ft.close()
    return {"mpps_median": round(n / (med / 1e3) / 1e6, 3), "launch_ms_median": round(med, 4),
            "lean_units": bool(lean),
            "full_units": {"mpps_median": round(n / (med_full / 1e3) / 1e6, 3),
                           "launch_ms_median": round(med_full, 4), "lean_units": bool(lean_f),
                           "what": "the same launches through the units an image with stateful NAT runs "
                                   "(port forwarding / masquerade compiled in; context tables in LDS)"},
            "flows": int((res == A.FLOW_INSERTED).sum()), "table_slots": slots,
            "insert_s": round(t_ins, 3), "packets_with_flow": hit, "flows_active_after": int(act),
            "what": "the same burst with a flow table attached: every other packet's flow pair "
                    "established (Active, current generation), FlowLookup on every overlay "
                    "packet, flow-filter bypass, flows-variant kernel + fix-up + invalidation "
                    "kernels per launch, dp_pkt_meta_t (flow refs) written "
                    "(median of %d launches)" % steps}


def nat_leg(dev, stream, steps: int, n: int, kind: str = "pf") -> dict:
    """Port forwarding under load: a burst of n 64-byte
    packets of which a share opens new port-forwarded connections
    (dataplane_amd/natwork.py), through the flows variant with its NAT pass
    (dp_nat_prep + dp_nat_resolve: one lane per connection) and replay; the
    table is emptied between launches (untimed), so every launch creates its
    connections anew.  The last line: the same at the largest share with the
    NAT pass forced onto one lane in packet order (the round-3 resolver).
    Reported beside `value`, never inside it."""
    from dataplane_amd import natwork as W
    from dataplane_amd.flows import FlowTable
    lib = A.gpu_lib()
    nf2 = GpuPathNf(dev.index)
    nf2.publish((W.masq_tables() if kind == "masq" else W.tables()).build())
    slots = 1 << max(12, int(np.ceil(np.log2(max(1, 4 * n)))))  # (8M for 2M packets: 1 GiB)
    ft = FlowTable(dev.index, slots)
    nf2.attach_flows(ft)
    sptr = stream.cuda_stream
    res = {"packets": n, "table_slots": slots, "legs": []}
    hour = 3600 * 10**9
    clock = [0]

    def counters():
        import ctypes as C
        c = (C.c_uint32 * 40)()
        lib.dpf_debug_nat_counters(nf2.ctx, c, 40)
        return {"mode": int(c[12]), "records": int(c[1]), "lane_records": int(c[11]),
                "connections": int(c[4]), "left_by_connections": int(c[13]), "allocations_batched": int(c[14]),
                "allocations_alone": int(c[15]), "lane_kticks": [int(c[19 + k]) for k in range(7)],
                "allocation_steps": int(c[26]), "steady_refreshes": bool(c[27]),
                "bulk_served_lane_records": int(c[35]), "bulk_blocks": int(c[39])}

    def run(share, reps, one_lane=False, near_capacity=False):
        buf, inp, npf = W.burst(n, share, 0, kind=kind)
        filled = 0
        if near_capacity:
            # the table pre-filled with flows that never expire, up to `npf`
            # slots below its capacity: half of the burst's pairs fit, the
            # rest are refused (insert_common's admissions, decided in packet
            # order before the connections run: mode 4)
            cap = min(10_000_000, slots // 2)  # FlowTable::DEFAULT_CAPACITY, at most half the slots
            ft.set_capacity(cap)
            clock[0] += hour
            ft.sweep(clock[0])  # (the last leg's flows gone)
            filled = max(0, cap - npf)
            fl = np.zeros(filled, A.FLOW)
            i = np.arange(filled, dtype=np.uint64)
            fl["key"]["src_vni"], fl["key"]["family"], fl["key"]["kind"] = W.VPC_P, 4, A.FLOW_UDP
            fl["key"]["sport"], fl["key"]["dport"] = 1000, 53
            fl["key"]["src"][:, :4] = W._ip((np.uint64(172 << 24 | 16 << 16) + i).astype(np.uint32))
            fl["key"]["dst"][:, :4] = (198, 51, 100, 1)
            fl["dst_vni"] = W.VPC_C
            fl["expires_at"] = (1 << 63) - 1
            for k in range(0, filled, 1 << 20):
                ft.insert(fl[k:k + (1 << 20)])
            log(0, f"[bench] NAT leg: table pre-filled with {filled} flows, capacity {cap}")
        pristine = torch.from_numpy(buf).to(dev)
        b = torch.empty_like(pristine)
        dinp = torch.from_numpy(inp.view(np.uint8)).to(dev)
        dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
        ms, flows = [], 0
        lib.dpf_debug_nat_sequential(1 if one_lane else 0)
        try:
            for k in range(reps):
                clock[0] += hour
                nf2.set_option(A.OPT_CLOCK, clock[0])
                ft.sweep(clock[0])  # every flow of the last launch expired: an empty table
                b.copy_(pristine)
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                nf2.process_device(b.data_ptr(), b.numel(), dinp.data_ptr(), dout.data_ptr(), n, None, sptr)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                ms.append(e0.elapsed_time(e1))
                flows = ft.count()[0]
        finally:
            lib.dpf_debug_nat_sequential(0)
        out = np.frombuffer(dout.cpu().numpy().tobytes(), dtype=A.PKT_OUT)
        done = {A.DONE_NAMES[d]: int(c) for d, c in zip(*np.unique(out["done"], return_counts=True))}
        keep = ms[1:] if len(ms) > 1 else ms
        med = sorted(keep)[len(keep) // 2]
        if filled:
            ft.remove(fl["key"])
        return {"pf_share": share, "pf_packets": npf, "one_lane": one_lane, "prefilled_flows": filled,
                "nat_pass": counters(), "launch_ms_median": round(med, 4),
                "mpps_median": round(n / (med / 1e3) / 1e6, 3), "flows_after": int(flows), "launches": len(keep),
                "done_histogram": done}

    def run_established(reps, conns=500_000, new_share=0.01, fwd_share=0.6):
        """Every packet masqueraded: `conns` connections opened by an untimed
        burst, then 2M-packet bursts of which 99 % belong to them (the
        clients' packets and the servers' answers to the public tuples,
        shuffled) and 1 % open new connections (fresh clients every launch)."""
        nf2.publish(W.masq_world().build())
        clock[0] += hour
        nf2.set_option(A.OPT_CLOCK, clock[0])
        ft.sweep(clock[0])
        c = W.MasqConns(conns)
        buf, inp = c.first()
        b = torch.from_numpy(buf).to(dev)
        dinp = torch.from_numpy(inp.view(np.uint8)).to(dev)
        dout = torch.empty(len(inp) * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
        nf2.process_device(b.data_ptr(), b.numel(), dinp.data_ptr(), dout.data_ptr(), len(inp), None, sptr)
        torch.cuda.synchronize(dev)
        out0 = np.frombuffer(dout.cpu().numpy().tobytes(), dtype=A.PKT_OUT)
        learnt = c.learn(b.cpu().numpy(), out0)
        ms, cnts, done = [], [], {}
        for k in range(reps):
            buf, inp, nn = c.burst(n, new_share, fwd_share, step=k + 1)
            b = torch.from_numpy(buf).to(dev)
            dinp = torch.from_numpy(inp.view(np.uint8)).to(dev)
            dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
            clock[0] += 10 ** 6
            nf2.set_option(A.OPT_CLOCK, clock[0])
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            nf2.process_device(b.data_ptr(), b.numel(), dinp.data_ptr(), dout.data_ptr(), n, None, sptr)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms.append(e0.elapsed_time(e1))
            cnts.append(counters())
            out = np.frombuffer(dout.cpu().numpy().tobytes(), dtype=A.PKT_OUT)
            done = {A.DONE_NAMES[d]: int(x) for d, x in zip(*np.unique(out["done"], return_counts=True))}
        keep = ms[1:] if len(ms) > 1 else ms
        med = sorted(keep)[len(keep) // 2]
        # every flow expires: the sweep drops them and gives their tuples back
        # (the release kernels, one lane per address record)
        flows_before = int(ft.count()[0])
        clock[0] += hour
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        swept = ft.sweep(clock[0])
        sweep_ms = (time.perf_counter() - t0) * 1e3
        return {"established_connections": conns, "learnt": learnt, "new_share": new_share,
                "sweep": {"flows": flows_before, "removed": int(swept) if swept is not None else None,
                          "ms": round(sweep_ms, 3),
                          "what": "dp_flow_sweep of every flow (expired), its allocations released"},
                "client_share": fwd_share, "launch_ms_median": round(med, 4), "launch_ms": [round(x, 4) for x in ms],
                "mpps_median": round(n / (med / 1e3) / 1e6, 3), "flows_after": int(ft.count()[0]),
                "launches": len(keep), "nat_pass": cnts[-1], "done_histogram": done}

    def run_mixed(reps, conns=250_000, new_share=0.02, one_lane=False):
        """Port forwarding and masquerade on one public range (natwork.
        mixed_world: the reference's overlapping-expose configuration):
        `conns` port-forwarded and `conns` masqueraded connections opened by
        an untimed burst, then 2M-packet bursts, 1 % new port-forwarded and
        1 % new masqueraded connections, the rest on the known ones (both
        sides, the answers included).  The first two timed bursts move the
        new pairs two-way and established; the median is over the rest."""
        clock[0] += hour
        nf2.set_option(A.OPT_CLOCK, clock[0])
        ft.sweep(clock[0])
        nf2.publish(W.mixed_world().build())
        c = W.MixedConns(conns, conns)
        buf, inp = c.first()
        b = torch.from_numpy(buf).to(dev)
        dinp = torch.from_numpy(inp.view(np.uint8)).to(dev)
        dout = torch.empty(len(inp) * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
        nf2.process_device(b.data_ptr(), b.numel(), dinp.data_ptr(), dout.data_ptr(), len(inp), None, sptr)
        torch.cuda.synchronize(dev)
        first = counters()
        out0 = np.frombuffer(dout.cpu().numpy().tobytes(), dtype=A.PKT_OUT)
        learnt = c.learn(b.cpu().numpy(), out0)
        ms, cnts, done = [], [], {}
        lib.dpf_debug_nat_sequential(4 if one_lane else 0)
        try:
            for k in range(reps):
                buf, inp, npf, nm = c.burst(n, new_share, step=k + 1)
                b = torch.from_numpy(buf).to(dev)
                dinp = torch.from_numpy(inp.view(np.uint8)).to(dev)
                dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
                clock[0] += 10 ** 6
                nf2.set_option(A.OPT_CLOCK, clock[0])
                torch.cuda.synchronize(dev)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                nf2.process_device(b.data_ptr(), b.numel(), dinp.data_ptr(), dout.data_ptr(), n, None, sptr)
                e1.record(stream)
                torch.cuda.synchronize(dev)
                ms.append(e0.elapsed_time(e1))
                cnts.append(counters())
                out = np.frombuffer(dout.cpu().numpy().tobytes(), dtype=A.PKT_OUT)
                done = {A.DONE_NAMES[d]: int(x) for d, x in zip(*np.unique(out["done"], return_counts=True))}
        finally:
            lib.dpf_debug_nat_sequential(0)
        keep = ms[2:] if len(ms) > 2 else ms
        med = sorted(keep)[len(keep) // 2]
        return {"connections": {"port_forwarded": conns, "masqueraded": conns, "learnt": learnt},
                "first_burst_nat_pass": first, "new_share": new_share, "one_lane": one_lane,
                "launch_ms_median": round(med, 4), "launch_ms": [round(x, 4) for x in ms],
                "mpps_median": round(n / (med / 1e3) / 1e6, 3), "flows_after": int(ft.count()[0]),
                "launches": len(keep), "nat_pass": cnts[-1], "done_histogram": done}

    if kind == "mixed":
        res["mixed"] = run_mixed(min(steps, 4) + 2)
        log(0, f"[bench] mixed leg (port forwarding + masquerade, 1 % + 1 % new): "
               f"{res['mixed']['launch_ms_median']} ms, mode {res['mixed']['nat_pass']['mode']}")
    elif kind == "masq":
        # first packets of new connections only (the allocating lane), then
        # every packet masqueraded (connection lanes + the allocating lane)
        for share in (0.001, 0.01):
            res["legs"].append(run(share, min(steps, 3) + 1))
            res["legs"][-1]["nat_pass"] = counters()
            log(0, f"[bench] masquerade leg share {share}: {res['legs'][-1]['launch_ms_median']} ms")
        res["established"] = run_established(min(steps, 4) + 1)
        log(0, f"[bench] masquerade leg, every packet masqueraded (99% established, 1% new): "
               f"{res['established']['launch_ms_median']} ms")
    else:
        for share in (0.0, 0.01, 0.05, 0.25):
            res["legs"].append(run(share, steps + 1))
            log(0, f"[bench] NAT leg share {share}: {res['legs'][-1]['launch_ms_median']} ms")
        res["legs"].append(run(0.25, 2, one_lane=True))
        log(0, f"[bench] NAT leg one lane: {res['legs'][-1]['launch_ms_median']} ms")
        res["legs"].append(run(0.25, steps + 1, near_capacity=True))
        log(0, f"[bench] NAT leg near capacity: {res['legs'][-1]['launch_ms_median']} ms")
    nf2.attach_flows(None)
    ft.close()
    nf2.close()
    res["what"] = ("flows variant with %s creations: first pass, NAT pass (dp_nat_prep + "
                   "dp_nat_resolve%s), replay, fix-up, invalidation, per launch (HIP events, median); "
                   "per-kernel times: profiles/ rocprofv3 stats of this leg"
                   % ({"masq": ("masquerade (allocations from a 256-address pool)", " + dp_nat_lane_order + dp_nat_lane"),
                       "mixed": ("port-forwarding and masquerade (one public /24, forwarded ports claimed)",
                                 " + dp_nat_cross + dp_nat_lane")}.get(kind, ("port-forwarding", ""))))
    return res


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list, port: int = 0) -> int:
    """`bench.py --gpus N` started without a launcher: start N rank processes of
    this same command line (one per GPU, RANK = LOCAL_RANK = i, WORLD_SIZE = N,
    rendezvous on 127.0.0.1), wait for all of them and return the worst exit
    status.  Runs before anything touches the GPU, and starts children rather
    than replacing this process.  The per-worker split it stands for is the
    reference's fan-out of one rx stream over N workers
    (dataplane/src/drivers/kernel/fanout.rs:49-73); here each rank is a GPU
    processing its own shard."""
    import subprocess
    port = port or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    worst = 0
    for p in procs:
        rc = p.wait()
        if rc != 0 and worst == 0:
            worst = rc if rc > 0 else 1
    return worst


def check_world(gpus: int, env=os.environ) -> int:
    """The world size this run will use; exits non-zero when --gpus and the
    launcher's WORLD_SIZE disagree (a run that would time another N)."""
    if "WORLD_SIZE" not in env:
        return 1
    world = int(env["WORLD_SIZE"])
    if world != gpus:
        print(f"bench.py: --gpus {gpus} but WORLD_SIZE={world} (launcher started {world} ranks)",
              file=sys.stderr, flush=True)
        sys.exit(2)
    return world


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--packets", type=int, default=2_000_000, help="packets per step per GPU")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-sample", type=int, default=500_000)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true")
    ap.add_argument("--no-flows", action="store_true", help="skip the flow-table leg")
    ap.add_argument("--no-nat", action="store_true", help="skip the port-forwarding (NAT pass) leg")
    ap.add_argument("--nat-only", action="store_true", help="only the NAT leg (profiling)")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N > 1: skip the resident-burst scatter / process / gather measurement")
    # ablation knobs (0 = the config's default table sizes)
    ap.add_argument("--routes-v4", type=int, default=0)
    ap.add_argument("--routes-v6", type=int, default=0)
    ap.add_argument("--acl", type=int, default=0)
    ap.add_argument("--nat", type=int, default=0)
    ap.add_argument("--layout", choices=["dpdk", "packed"], default="dpdk",
                    help="burst buffer layout: DPDK mbuf data (128 B headroom, 64-byte aligned "
                         "frames) or packed (96 B headroom, 16-byte aligned)")
    ap.add_argument("--nat-kind", choices=["both", "pf", "masq", "mixed"], default="both",
                    help="with --nat-only: which NAT legs")
    ap.add_argument("--launch-probe", action="store_true",
                    help="test hook: each rank prints its rank / world as JSON and exits before "
                         "any GPU call")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks ourselves (before any GPU call)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = check_world(args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_probe:
        print(json.dumps({"rank": rank, "local_rank": local, "world": world,
                          "master": os.environ.get("MASTER_ADDR")}), flush=True)
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        import datetime
        # a hung collective ends the run in minutes, not the 10-minute default
        dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=180))

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    if args.nat_only:  # the NAT legs alone (rocprofv3 of their kernels)
        st = torch.cuda.Stream(dev)
        legs = {}
        if args.nat_kind in ("both", "pf"):
            legs["nat_portfw"] = nat_leg(dev, st, min(args.steps, 10), args.packets)
        if args.nat_kind in ("both", "masq"):
            legs["nat_masquerade"] = nat_leg(dev, st, min(args.steps, 10), args.packets, kind="masq")
        if args.nat_kind in ("both", "mixed"):
            legs["nat_mixed"] = nat_leg(dev, st, min(args.steps, 10), args.packets, kind="mixed")
        print(json.dumps(legs), flush=True)
        return
    cfg = args.config
    t0 = time.perf_counter()
    w = Workload(cfg, args.packets, seed=shard_seed(args.seed, rank), n_routes_v4=args.routes_v4,
                 n_routes_v6=args.routes_v6, n_acl=args.acl, n_nat=args.nat, layout=args.layout)
    log(rank, f"[bench] workload C{cfg}: {w.n} packets, built in {time.perf_counter() - t0:.1f}s")
    nf = GpuPathNf(local)
    t0 = time.perf_counter()
    nf.publish(w.tables)
    log(rank, f"[bench] tables published in {time.perf_counter() - t0:.1f}s, "
              f"{nf.device_table_bytes() / 2**20:.1f} MiB device image")

    n = w.n
    bb = (w.buf.nbytes + 255) & ~255
    nbuf = args.warmup + args.steps
    pristine = torch.from_numpy(w.buf).to(dev)
    bufs = torch.empty((nbuf, bb), dtype=torch.uint8, device=dev)
    for k in range(nbuf):
        bufs[k, :w.buf.nbytes].copy_(pristine)
    dinp = torch.from_numpy(w.inp.view(np.uint8)).to(dev)
    dout = torch.empty(n * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
    dstats = torch.zeros(A.DONE_COUNT, dtype=torch.int64, device=dev)
    # a dedicated (non-default) stream: the kernel and the timing events must
    # share it (the default stream's handle is 0, which the ABI maps to the
    # context's own stream)
    stream = torch.cuda.Stream(dev)
    sptr = stream.cuda_stream
    torch.cuda.synchronize(dev)

    def step(k):
        nf.process_device(bufs[k].data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n,
                          dstats.data_ptr(), sptr)

    for k in range(args.warmup):
        step(k)
    torch.cuda.synchronize(dev)
    dstats.zero_()
    # one event per step boundary, on the launch stream: per-step durations
    # (median) besides the whole timed region
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        step(args.warmup + k)
        evs[k + 1].record(stream)
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t_start
    step_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
    kernel_ms = evs[0].elapsed_time(evs[-1]) / args.steps

    # roofline timing of dp_pipeline_kernel alone (no histogram, so no
    # dp_stats_reduce launch): one event pair per launch, re-using the
    # processed buffers' pristine copies
    for k in range(nbuf):
        bufs[k, :w.buf.nbytes].copy_(pristine)
    torch.cuda.synchronize(dev)
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    for k in range(args.steps):
        kev[k][0].record(stream)
        nf.process_device(bufs[args.warmup + k].data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n,
                          None, sptr)
        kev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    launch_ms = sorted(a.elapsed_time(b) for a, b in kev)
    pipe_ms_median = launch_ms[len(launch_ms) // 2]
    pipe_ms_mean = sum(launch_ms) / len(launch_ms)
    # the same launches also writing the optional dp_pkt_meta_t array (the
    # rest of PacketMeta: VNIs, FIB entry, ACL rule, VRF, next hop, DSCP)
    dmeta = torch.empty(n * A.PKT_META.itemsize, dtype=torch.uint8, device=dev)
    for k in range(nbuf):
        bufs[k, :w.buf.nbytes].copy_(pristine)
    torch.cuda.synchronize(dev)
    for k in range(args.steps):
        kev[k][0].record(stream)
        nf.process_device(bufs[args.warmup + k].data_ptr(), bb, dinp.data_ptr(), dout.data_ptr(), n,
                          None, sptr, dev_meta=dmeta.data_ptr())
        kev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    meta_ms = sorted(a.elapsed_time(b) for a, b in kev)
    meta_ms_median = meta_ms[len(meta_ms) // 2]
    del dmeta

    elapsed, hist = reduce_over_ranks(elapsed, dstats.cpu().numpy(), dev)

    # N > 1, after the timed region: the path for a burst resident on one GPU
    # (rank 0's shard scattered over all ranks with RCCL point-to-point sends,
    # processed, gathered back), reported beside -- never inside -- `value`
    rccl = None
    if world > 1 and not args.no_rccl:
        del bufs
        w0 = w if rank == 0 else Workload(cfg, args.packets, seed=shard_seed(args.seed, 0),
                                          n_routes_v4=args.routes_v4, n_routes_v6=args.routes_v6,
                                          n_acl=args.acl, n_nat=args.nat, layout=args.layout)

        def process_shard(span, rin, cnt):
            o = torch.empty(max(1, cnt) * A.PKT_OUT.itemsize, dtype=torch.uint8, device=dev)
            if cnt:
                nf.process_device(span.data_ptr(), span.numel(), rin.data_ptr(), o.data_ptr(), cnt,
                                  None, sptr)
            return o
        rccl = timed_scatter_gather(w0.inp, w0.fresh_buf, process_shard, rank, world, dev,
                                    A.PKT_IN.itemsize, A.PKT_OUT.itemsize)

    ms_per_step = elapsed * 1e3 / args.steps
    total_pkts = world * n * args.steps
    value = total_pkts / elapsed / 1e6
    delivered = int(hist[A.DONE["Delivered"]])
    # (DP_BENCH_NOCHECK: diagnostic builds with stages compiled out deliver nothing)
    if int(hist.sum()) != total_pkts or (delivered == 0 and not os.environ.get("DP_BENCH_NOCHECK")):
        raise RuntimeError(f"bad DoneReason histogram: {hist.tolist()}")

    result = None
    if rank == 0:
        achieved = n * ALGO_BYTES[cfg] / (pipe_ms_mean / 1e3) / 1e9
        traffic, traffic_src = measured_traffic(cfg, n)
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                    "kernel": "dp_pipeline_kernel", "kernel_ms": round(pipe_ms_mean, 4),
                    "kernel_ms_median": round(pipe_ms_median, 4),
                    "kernel_timing": f"HIP events around each of {args.steps} launches on the "
                                     "launch stream (achieved uses the mean, as rocprof's "
                                     "AverageNs)",
                    "bytes_per_pkt": ALGO_BYTES[cfg]}
        if traffic is not None:
            roofline["traffic_unit"] = "bytes per launch"
            roofline["traffic_source"] = traffic_src
        result = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mpps", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded, SURVEY.md §8d)",
            "config": {"workload": f"C{cfg}: " + CONFIG_NAMES[cfg], "packets_per_step_per_gpu": n,
                       "frame_bytes_per_step_per_gpu": w.frame_bytes, "seed": args.seed,
                       "buffer_layout": args.layout,
                       "table_overrides": {k: v for k, v in dict(routes_v4=args.routes_v4,
                                           routes_v6=args.routes_v6, acl=args.acl,
                                           nat=args.nat).items() if v},
                       "parallelism": f"dp{world} (independent shards)"},
            "step_ms_median": round(sorted(step_ms)[len(step_ms) // 2], 4),
            "step_ms_events_mean": round(kernel_ms, 4),
            "mpps_median_step": round(world * n / (sorted(step_ms)[len(step_ms) // 2] / 1e3) / 1e6, 3),
            "roofline": roofline,
            "with_meta": {"kernel_ms_median": round(meta_ms_median, 4),
                          "mpps_median": round(n / (meta_ms_median / 1e3) / 1e6, 3),
                          "what": "the same launches also writing dp_pkt_meta_t (48 B per "
                                  "packet: the rest of PacketMeta) beside dp_pkt_out_t"},
            "done_histogram": {A.DONE_NAMES[i]: int(c) for i, c in enumerate(hist) if c},
        }
        if rccl:
            result["resident_burst_scatter_gather"] = rccl
        if world == 1 and not args.no_flows:
            result["flow_table"] = flows_leg(nf, w, dev, stream, args.steps)
        if world == 1 and not args.no_nat:
            result["nat_portfw"] = nat_leg(dev, stream, min(args.steps, 10), n)
            result["nat_masquerade"] = nat_leg(dev, stream, min(args.steps, 10), n, kind="masq")
            result["nat_mixed"] = nat_leg(dev, stream, min(args.steps, 10), n, kind="mixed")
        if world == 1 and not args.no_host:
            # host-origin rate (dp_process_burst): pinned host burst buffer and
            # records, chunked H2D / kernel / D2H overlapped on several streams
            def pinned(nbytes):
                return torch.empty(nbytes, dtype=torch.uint8).pin_memory().numpy()
            pnp = pinned(w.buf.nbytes)
            pin_in = pinned(w.inp.nbytes).view(A.PKT_IN)
            pin_in[:] = w.inp
            pin_out = pinned(n * A.PKT_OUT.itemsize).view(A.PKT_OUT)
            def time_host(mode, reps=5):
                nf.set_host_path(mode)
                t_host = []
                for r in range(reps + 1):
                    pnp[:] = w.buf
                    t0 = time.perf_counter()
                    nf.process_arrays(pnp, pin_in, out=pin_out, with_meta=False)
                    if r > 0:
                        t_host.append(time.perf_counter() - t0)
                return sorted(t_host)[len(t_host) // 2]
            th = time_host(A.HOST_COPY)
            # what crosses PCIe: each frame's 16-byte span in (+ its position)
            # and out (+ the 96 B headroom where routes encapsulate: C4), the
            # in / out records
            off = w.inp["off"].astype(np.int64)
            span = int((((off + w.inp["len"] + 15) >> 4) - (off >> 4)).sum()) * 16
            grow = 96 * n if w.config == 4 else 0
            pcie_bytes = 2 * span + grow + n * (A.PKT_IN.itemsize + A.PKT_OUT.itemsize + 4)
            host = {"mpps_median": round(n / th / 1e6, 3), "runs": 5,
                    "pcie_bytes_per_burst": pcie_bytes,
                    "pcie_bytes_per_pkt": round(pcie_bytes / n, 1),
                    "pcie_gbs": round(pcie_bytes / th / 1e9, 2),
                    "what": "dp_process_burst on pinned host buffers, staged copies: host "
                            "threads pack the frames' 16-byte spans, spans + records H2D, "
                            "kernel, packed spans + records D2H, frames written back in "
                            "place; chunks of 64K+ packets on 3 streams"}
            try:
                tz = time_host(A.HOST_ZERO_COPY)
                host["zero_copy"] = {
                    "mpps_median": round(n / tz / 1e6, 3),
                    "what": "dp_process_burst with DP_HOST_ZERO_COPY: the kernel reads and "
                            "rewrites the frames in mapped pinned host memory over PCIe, no "
                            "staging copies"}
            except RuntimeError as e:
                host["zero_copy"] = {"error": str(e)}
            nf.set_host_path(A.HOST_AUTO)
            best = max(host["mpps_median"], host.get("zero_copy", {}).get("mpps_median", 0))
            result["host_inclusive_mpps"] = best
            result["host_inclusive"] = host
        if world == 1 and not args.no_cpu:
            result["cpu_baseline"] = cpu_baseline(w, args.cpu_sample, args.cpu_budget)
        print(json.dumps(result), flush=True)
    nf.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
