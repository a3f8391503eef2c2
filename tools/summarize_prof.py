#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC
passes) into profiles/<tag>_*.json / .md.

HBM traffic per launch follows MI355X_MICROARCH.md §HBM for gfx950: FETCH_SIZE reports
exactly half the bytes of a wide coalesced streaming read (16 B/lane loads), so it is
doubled; WRITE_SIZE reads exactly for 16-B-per-lane streaming stores.  Both counters are in
KiB (1024 B).
"""
import argparse
import csv
import json
import os
import statistics


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True, help="dir with *_kernel_stats.csv")
    ap.add_argument("--fetch", help="dir with the FETCH_SIZE pmc_counter_collection.csv")
    ap.add_argument("--write", help="dir with the WRITE_SIZE pmc_counter_collection.csv")
    ap.add_argument("--kernel", required=True, help="substring of the kernel name")
    ap.add_argument("--algo-bytes", type=float, required=True, help="algorithmic bytes/launch")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--out", default="profiles")
    a = ap.parse_args()
    import glob
    ks = sorted(glob.glob(os.path.join(a.trace, "**", "*kernel_stats.csv"), recursive=True))
    if not ks:
        raise SystemExit(f"no *kernel_stats.csv under {a.trace}")
    stats = [r for r in rows(ks[0])]
    k = [r for r in stats if a.kernel in r["Name"]]
    if not k:
        raise SystemExit("kernel not found in stats")
    k = k[0]
    res = {"kernel": k["Name"], "calls": int(k["Calls"]), "avg_ns": float(k["AverageNs"]),
           "min_ns": float(k["MinNs"]), "max_ns": float(k["MaxNs"]),
           "algorithmic_bytes_per_launch": a.algo_bytes}
    res["algorithmic_GBps_at_avg"] = a.algo_bytes / res["avg_ns"]
    if a.fetch and a.write:
        f = [float(r["Counter_Value"]) for r in rows(os.path.join(a.fetch, "pmc_counter_collection.csv"))
             if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
        w = [float(r["Counter_Value"]) for r in rows(os.path.join(a.write, "pmc_counter_collection.csv"))
             if a.kernel in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE"]
        fetch_b = 2.0 * statistics.median(f) * 1024.0
        write_b = statistics.median(w) * 1024.0
        res.update({"FETCH_SIZE_KiB_median": statistics.median(f), "WRITE_SIZE_KiB_median": statistics.median(w),
                    "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
                    "hbm_bytes_per_launch": fetch_b + write_b,
                    "traffic_over_algorithmic": (fetch_b + write_b) / a.algo_bytes,
                    "pmc_launches": [len(f), len(w)]})
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, a.tag + ".json"), "w") as fo:
        json.dump(res, fo, indent=1)
    # human-readable copy of the stats table
    with open(os.path.join(a.out, a.tag + "_kernel_stats.md"), "w") as fo:
        fo.write("| kernel | calls | avg us | min us | max us | % |\n|---|---|---|---|---|---|\n")
        for r in stats[:15]:
            fo.write(f"| {r['Name'][:90]} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                     f"{float(r['MinNs'])/1e3:.1f} | {float(r['MaxNs'])/1e3:.1f} | {r['Percentage']} |\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
