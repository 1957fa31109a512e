#!/usr/bin/env python3
"""Summarise scripts/profile_bf16.sh output: per bf16 shape the fold kernel's
rocprofv3 time per fold call (band dispatches summed), algorithmic GB/s, the
in-run read-sweep ceiling, HBM bytes / algorithmic bytes (FETCH_SIZE x 2 x
1 KiB + WRITE_SIZE x 1 KiB, gfx950 corrections of MI355X_MICROARCH.md), and
SQ_WAIT_ANY / SQ_WAVE_CYCLES; then C5's FETCH / WRITE traffic.

    python scripts/bf16_summary.py gpurun_out/bf16 > profiles/r03_bf16/SUMMARY.md
"""
import csv
import glob
import json
import os
import statistics
import sys


def counters(d, kernel):
    agg = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"]:
                agg.setdefault(row["Counter_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                agg[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in agg.items()}


def main():
    root = sys.argv[1]
    print("| clients x params (bf16) | fold kernel | dispatches / call | rocprof ms / call | algorithmic GB/s | "
          "frac of 8 TB/s | read sweep GB/s (same bytes) | frac of sweep | HBM / algorithmic | "
          "SQ_WAIT_ANY / SQ_WAVE_CYCLES | VALU insts / VMEM rd insts |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for d in sorted(glob.glob(os.path.join(root, "n*_p*"))):
        tag = os.path.basename(d)
        n, p = (int(x) for x in tag[1:].split("_p"))
        alg = n * p * 2 + p * 4 + p * 2  # bf16 rows + fp32 result + its RNE bf16 copy
        line = json.loads(open(os.path.join(d, "bench.json")).read())
        stats = glob.glob(os.path.join(d, "trace", "*kernel_stats.csv"))[0]
        rows = [r for r in csv.DictReader(open(stats)) if "k_fedavg_bf16" in r["Name"]]
        r = rows[0]
        name = r["Name"][r["Name"].index("k_fedavg_bf16"):r["Name"].index(">") + 1]
        calls = line["steps"] + line["warmup"]
        dpc = round(int(r["Calls"]) / calls)
        ms = float(r["AverageNs"]) * dpc / 1e6
        c = counters(d, "k_fedavg_bf16")
        fetch = statistics.median(c["FETCH_SIZE"]) * dpc * 2 * 1024 if "FETCH_SIZE" in c else float("nan")
        write = statistics.median(c["WRITE_SIZE"]) * dpc * 1024 if "WRITE_SIZE" in c else 0.0
        wait = statistics.median(a / b for a, b in zip(c["SQ_WAIT_ANY"], c["SQ_WAVE_CYCLES"]))
        valu = statistics.median(a / b for a, b in zip(c["SQ_INSTS_VALU"], c["SQ_INSTS_VMEM_RD"]))
        sweep = line["roofline"]["read_sweep_ceiling"]
        gbs = alg / ms / 1e6
        print(f"| {n} x {p:,} | `{name}` | {dpc} | {ms:.3f} | {gbs:.0f} | {gbs / 8000:.3f} | {sweep:.0f} | "
              f"{gbs / sweep:.3f} | {(fetch + write) / alg:.4f} | {wait:.2f} | {valu:.1f} |")
    c5 = os.path.join(root, "c5")
    if os.path.isdir(c5):
        c = counters(c5, "k_fold_f32")
        n, p = 512, 25_000_000
        alg = n * p * 4 + p * 4
        # C5: fold calls = warmup 1 + steps 3 + the bench's extras are not folds; bands per call from the count
        per_call = len(c["FETCH_SIZE"]) // 4
        fetch = statistics.median(c["FETCH_SIZE"]) * per_call * 2 * 1024
        write = statistics.median(c["WRITE_SIZE"]) * per_call * 1024
        print()
        print(f"C5 (512 x 25M fp32 stall-aware): {per_call} band dispatches per call; HBM read "
              f"{fetch / 1e9:.3f} GB + write {write / 1e9:.4f} GB per call against {alg / 1e9:.3f} GB "
              f"algorithmic: ratio {(fetch + write) / alg:.4f}")


if __name__ == "__main__":
    main()
