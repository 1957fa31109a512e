#!/usr/bin/env python3
"""Summarise bench.py --sweep logs (<N>x<P>.log: 'variant k name median t ms'):
per shape the best form and the auto fold's ratio to it, then every form's
mean / worst ratio to the per-shape best.

    python scripts/sweep_summary.py DIR > DIR/SUMMARY.md
"""
import collections
import glob
import os
import re
import sys


def load(d):
    T = {}
    for f in glob.glob(os.path.join(d, "*.log")):
        m = re.match(r"(\d+)x(\d+)\.log$", os.path.basename(f))
        if not m:
            continue
        row = {}
        for line in open(f):
            mm = re.match(r"variant (\d+) (\S+)\s+median ([\d.]+) ms", line)
            if mm:
                # the product's auto fold is "auto" (fp32) or "bf16auto" (bf16)
                row["auto" if mm.group(2) == "bf16auto" else mm.group(2)] = float(mm.group(3))
        if row:
            T[(int(m.group(1)), int(m.group(2)))] = row
    return T


def main():
    d = sys.argv[1]
    T = load(d)
    print(f"# Sweep summary: {d}\n")
    print("| clients x params | best form | best ms | auto ms | auto / best |")
    print("|---|---|---|---|---|")
    agg = collections.defaultdict(list)
    for (n, p), row in sorted(T.items()):
        best_name = min(row, key=row.get)
        best = row[best_name]
        for k, v in row.items():
            agg[k].append(v / best)
        print(f"| {n} x {p:,} | {best_name} | {best:.4f} | {row.get('auto', float('nan')):.4f} | "
              f"{row.get('auto', float('nan')) / best:.3f} |")
    print("\n| form | mean ratio to best | worst | shapes |")
    print("|---|---|---|---|")
    for k, r in sorted(agg.items(), key=lambda kv: sum(kv[1]) / len(kv[1])):
        print(f"| {k} | {sum(r) / len(r):.3f} | {max(r):.3f} | {len(r)} |")


if __name__ == "__main__":
    main()
