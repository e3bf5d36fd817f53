"""The CPU baseline as BASELINE.md plans it (BASELINE.md:37-55), beside the
bounded sample bench.py reports: per config C1-C5, the median of >= 20 runs
of >= 10M packets each on one thread per physical core of the job's CPU share,
plus a 1-thread figure, for two legs:

  - "port": the oracle (oracle/), the C++ restatement of the reference
    pipeline with the reference's own classifier shapes (linear-scan ACL and
    flow-filter rules, a binary-trie LPM) -- the reference's CPU pipeline;
  - "compiled": the kernel's per-packet body built for the host (tests/emu,
    -O3) over the same compiled table image (Poptrie / DIR-24-8 LPM,
    candidate-list classifiers): the fair classifier baseline, the data
    structures a tuned CPU build would use.

A run of N packets is N / burst passes over the config's seeded 2M-packet
burst, each over a fresh copy of its frames (the path rewrites them), in
bursts of 64.  CPU only; run it on the GPU box's host cores:

    python scripts/cpu_baseline_plan.py --configs 1 2 3 --out gpurun_out/cpu_plan_a.json

Test infrastructure: the oracle is the measured baseline here, never the
product path."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "emu"))

from dataplane_amd import _abi as A  # noqa: E402
from dataplane_amd.workload import CONFIG_NAMES, Workload  # noqa: E402


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def runs(process, w: Workload, n_run: int, reps: int, tag: str = "") -> list:
    """reps timed runs of n_run packets (passes over the burst); Mpps each
    (one progress line per run: a long silent run reads as hung)"""
    out = []
    inp = w.inp.copy()
    res = np.zeros(w.n, dtype=A.PKT_OUT)
    for _ in range(reps):
        done, t = 0, 0.0
        while done < n_run:
            m = min(w.n, n_run - done)
            buf = w.fresh_buf()
            t0 = time.perf_counter()
            process(buf, inp[:m], res[:m])
            t += time.perf_counter() - t0
            done += m
        out.append(done / t / 1e6)
        print(f"[cpu-plan] {tag} run {len(out)}/{reps}: {out[-1]:.4f} Mpps", flush=True)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2, 3, 4, 5])
    ap.add_argument("--packets", type=int, default=10_000_000, help="packets per run")
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--one-thread-packets", type=int, default=1_000_000)
    ap.add_argument("--one-thread-runs", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    bm = _bench()
    threads = bm.cpu_threads()
    from oracle.pyoracle import Oracle  # test-infrastructure checker, timed as the baseline
    import pyemu  # test infrastructure (host build of the kernel body)
    result = {"what": "BASELINE.md CPU plan: median of >= 20 runs of >= 10M packets per config, "
                      "bursts of 64, one thread per physical core of the job's CPU share; "
                      "1-thread figures over fewer, shorter runs",
              "cpu_model": bm.cpu_model(), "threads": threads,
              "runs": args.runs, "packets_per_run": args.packets, "configs": {}}
    for cfg in args.configs:
        t0 = time.perf_counter()
        w = Workload(cfg, 2_000_000, seed=1)
        print(f"[cpu-plan] C{cfg}: workload in {time.perf_counter() - t0:.1f}s", flush=True)
        entry = {"workload": CONFIG_NAMES[cfg]}
        o = Oracle(w.tables)

        def port(th):
            return lambda buf, inp, out: o.process_parallel(buf, inp, out, threads=th, burst=64)
        t0 = time.perf_counter()
        pr = runs(port(threads), w, args.packets, args.runs, f"C{cfg} port")
        p1 = runs(port(1), w, args.one_thread_packets, args.one_thread_runs, f"C{cfg} port 1-thread")
        o.close()
        entry["port"] = {"median_mpps": round(statistics.median(pr), 4), "min": round(min(pr), 4),
                         "max": round(max(pr), 4), "runs": len(pr), "threads": threads,
                         "one_thread_median_mpps": round(statistics.median(p1), 4),
                         "one_thread_runs": f"{len(p1)} x {args.one_thread_packets}",
                         "seconds": round(time.perf_counter() - t0, 1),
                         "what": "the oracle: the reference pipeline's CPU restatement "
                                 "(linear-scan classifiers, binary-trie LPM)"}
        print(f"[cpu-plan] C{cfg} port {entry['port']}", flush=True)
        emu = pyemu.ParallelEmu(w.tables)
        ebuf = pyemu.aligned_copy(w.buf)

        def compiled(th):
            def run(buf, inp, out):
                ebuf[:buf.nbytes] = buf
                emu.run(ebuf, buf.nbytes, inp, out, threads=th, burst=64)
            return run
        t0 = time.perf_counter()
        cr = runs(compiled(threads), w, args.packets, args.runs, f"C{cfg} compiled")
        c1 = runs(compiled(1), w, args.one_thread_packets, args.one_thread_runs, f"C{cfg} compiled 1-thread")
        emu.close()
        entry["compiled"] = {"median_mpps": round(statistics.median(cr), 4), "min": round(min(cr), 4),
                             "max": round(max(cr), 4), "runs": len(cr), "threads": threads,
                             "one_thread_median_mpps": round(statistics.median(c1), 4),
                             "one_thread_runs": f"{len(c1)} x {args.one_thread_packets}",
                             "seconds": round(time.perf_counter() - t0, 1),
                             "what": "fair classifier baseline: the kernel's per-packet body "
                                     "compiled for the host (-O3, x86-64-v3) over the same table "
                                     "image (Poptrie / DIR-24-8 LPM, candidate-list classifiers)"}
        print(f"[cpu-plan] C{cfg} compiled {entry['compiled']}", flush=True)
        result["configs"][f"C{cfg}"] = entry
        if args.out:
            with open(args.out, "w") as f:
                json.dump(result, f, indent=1)
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
