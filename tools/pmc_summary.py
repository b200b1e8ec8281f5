#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/.

Per launch of mi_cls_kernel: the kernel-trace average duration and the PMC
counters.  HBM traffic is corrected as MI355X_MICROARCH.md (HBM section)
prescribes for gfx950:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x 1024);
  * FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced
    streaming read -> doubled (the kernel's packet-window loads are 16 B/lane
    buffer loads);
  * WRITE_SIZE is exact for 16 B/lane streaming stores (the result records).
Usage: tools/pmc_summary.py <gpurun_out/prof_TAG_cC> <tag> <workload key>
(workload key e.g. config3_n1000000, the key bench.py looks up).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(src, kernel="mi_cls_kernel"):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(src, "p*", "p_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def main():
    src, tag, key = sys.argv[1], sys.argv[2], sys.argv[3]
    ctr = counters(src)
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))):
        stats[r["Name"]] = {k: r[k] for k in ("Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
    name, k = [(n, v) for n, v in stats.items() if "mi_cls_kernel" in n][0]
    fetch, write = ctr["FETCH_SIZE"][0], ctr["WRITE_SIZE"][0]
    traffic = (2.0 * fetch + write) * 1024.0
    out = {
        "tag": tag, "workload": key,
        "kernel": name,
        "kernel_avg_ns": float(k["AverageNs"]), "kernel_calls": int(k["Calls"]),
        "FETCH_SIZE_KiB_per_launch": fetch, "WRITE_SIZE_KiB_per_launch": write,
        "hbm_bytes_per_launch": traffic,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count)",
        "counters_per_launch": {c: v for c, (v, _) in sorted(ctr.items())},
        "counter_launches": {c: n for c, (_, n) in sorted(ctr.items())},
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
              "SQ_INSTS_VALU_per_launch": ctr.get("SQ_INSTS_VALU", (None,))[0],
              "source": f"profiles/{tag}_pmc_{key}.json"}
    with open(p, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps({"traffic": traffic, "kernel_avg_ns": k["AverageNs"],
                      "valu": ctr.get("SQ_INSTS_VALU", (None,))[0]}))


if __name__ == "__main__":
    main()
