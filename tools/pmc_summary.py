#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/.

HBM traffic per launch of mi_cls_kernel from the PMC passes, corrected as
MI355X_MICROARCH.md (HBM section) prescribes for gfx950:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x 1024);
  * FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced
    streaming read -> doubled (the kernel's packet-window and descriptor
    loads are 16 B/lane / coalesced dword loads);
  * WRITE_SIZE is exact for 16 B/lane streaming stores (the result records).
Usage: tools/pmc_summary.py <gpurun_out/prof_TAG> <tag> <config key>
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(path, kernel="mi_cls_kernel"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"]]
    return sum(vals) / len(vals), len(vals)


def main():
    src, tag, key = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, nf = mean_counter(os.path.join(src, "fetch", "fetch_counter_collection.csv"))
    write, nw = mean_counter(os.path.join(src, "write", "write_counter_collection.csv"))
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
        stats[r["Name"]] = {k: r[k] for k in ("Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
    k = [v for n, v in stats.items() if "mi_cls_kernel" in n][0]
    traffic = (2.0 * fetch + write) * 1024.0
    out = {
        "tag": tag, "workload": key,
        "kernel": "mi_cls_kernel",
        "kernel_avg_ns": float(k["AverageNs"]), "kernel_calls": int(k["Calls"]),
        "FETCH_SIZE_KiB_per_launch": fetch, "WRITE_SIZE_KiB_per_launch": write,
        "pmc_launches": [nf, nw],
        "hbm_bytes_per_launch": traffic,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)",
        "kernel_stats": stats,
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{tag}_pmc_{key}.json"), "w") as f:
        json.dump(out, f, indent=1)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"),
                os.path.join(ROOT, "profiles", f"{tag}_kernel_stats_{key}.csv"))
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(p)) if os.path.exists(p) else {}
    d[key] = {"hbm_bytes_per_launch": traffic, "kernel_avg_ns": float(k["AverageNs"]),
              "source": f"profiles/{tag}_pmc_{key}.json"}
    with open(p, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps({"traffic": traffic, "kernel_avg_ns": k["AverageNs"]}))


if __name__ == "__main__":
    main()
