"""profiles/traffic.json from a gpu_pmc_all.sh run: per config, the measured
HBM bytes per packet of dp_pipeline_kernel<false, false, ...> (FETCH_SIZE x2,
WRITE_SIZE as read: MI355X_MICROARCH.md's gfx950 correction), for bench.py's
roofline.traffic.
    python scripts/traffic_json.py gpurun_out/pmcall profiles/r03/pmc_<sha>"""
import json
import os
import shutil
import sys

ALG = {1: 136.0, 2: 136.0, 3: 715.7, 4: 236.0, 5: 144.0}  # DESIGN.md §3 roofline


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    out = {}
    for c in range(1, 6):
        d = os.path.join(src, f"c{c}")
        if not os.path.exists(os.path.join(d, "summary.json")):
            continue
        s = json.load(open(os.path.join(d, "summary.json")))["derived"]
        shutil.copy(os.path.join(d, "summary.json"), os.path.join(dst, f"c{c}_pmc.json"))
        shutil.copy(os.path.join(d, "stats", "run_kernel_stats.csv"), os.path.join(dst, f"c{c}_kernel_stats.csv"))
        shutil.copy(os.path.join(d, "bench.json"), os.path.join(dst, f"c{c}_bench.json"))
        b = s["fetch_bytes_per_pkt_x2"] + s["write_bytes_per_pkt"]
        out[f"C{c}"] = {
            "bytes_per_pkt": round(b, 1),
            "fetch_bytes_per_pkt": s["fetch_bytes_per_pkt_x2"],
            "write_bytes_per_pkt": s["write_bytes_per_pkt"],
            "l2_hit": s.get("l2_hit"),
            "packets_per_launch_measured": 2000000,
            "source": f"{dst}/c{c}_pmc.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT_sum "
                      "TCC_MISS_sum, separate passes; dp_pipeline_kernel<false, false, false, *> dispatches only)",
            "correction": "FETCH_SIZE doubled, WRITE_SIZE as read (MI355X_MICROARCH.md, HBM section); KB units x1024",
            "traffic_over_algorithmic": round(b / ALG[c], 2),
        }
    json.dump(out, open(os.path.join("profiles", "traffic.json"), "w"), indent=1)
    print(json.dumps({k: v["bytes_per_pkt"] for k, v in out.items()}))


if __name__ == "__main__":
    main()
