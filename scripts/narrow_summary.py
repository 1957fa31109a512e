#!/usr/bin/env python3
"""Summarise scripts/profile_narrow.sh output (kernel stats + SQ / FETCH_SIZE
passes) into one markdown table: kernel-only time from rocprofv3, algorithmic
GB/s, HBM bytes / algorithmic bytes (FETCH_SIZE x 2 x 1 KiB, gfx950), and
SQ_WAIT_ANY / SQ_WAVE_CYCLES.

    python scripts/narrow_summary.py DIR [DIR ...] > SUMMARY.md
"""
import csv
import glob
import os
import statistics
import sys


def first(pattern):
    f = glob.glob(pattern)
    return f[0] if f else None


def main():
    print("| clients x params | fold kernel | rocprof avg us | algorithmic GB/s | frac of 8 TB/s | "
          "HBM bytes / algorithmic | SQ_WAIT_ANY / SQ_WAVE_CYCLES | waves |")
    print("|---|---|---|---|---|---|---|---|")
    for d in sys.argv[1:]:
        tag = os.path.basename(d.rstrip("/"))
        n, p = tag[1:].split("_p")
        n, p = int(n), int(p)
        alg = n * p * 4 + p * 4
        stats = first(os.path.join(d, "*kernel_stats.csv")) or first(os.path.join(d, "*", "*kernel_stats.csv"))
        rows = [r for r in csv.DictReader(open(stats)) if "k_fold" in r["Name"]]
        r = rows[0]
        name = r["Name"]
        name = name[name.index("k_fold"):name.index(">") + 1]
        ns = float(r["AverageNs"])
        agg = {}
        for f in glob.glob(os.path.join(d, "**", "*counter*.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "k_fold" in row["Kernel_Name"]:
                    agg.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        m = {k: statistics.median(v) for k, v in agg.items()}
        traffic = 2 * m["FETCH_SIZE"] * 1024 / alg if "FETCH_SIZE" in m else float("nan")
        wait = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"] if "SQ_WAIT_ANY" in m else float("nan")
        print(f"| {n} x {p:,} | `{name}` | {ns / 1e3:.1f} | {alg / ns:.0f} | {alg / ns / 8000:.3f} | "
              f"{traffic:.3f} | {wait:.2f} | {int(m.get('SQ_WAVES', 0))} |")


if __name__ == "__main__":
    main()
