#!/usr/bin/env python3
"""Per-round timeline of an end-to-end run (rocprofv3 --kernel-trace
--memory-copy-trace of bench_e2e.py): rounds are split at idle gaps of more
than 1 ms; per round the span from the first H2D to the result's D2H, the
H2D busy time and rate, the gaps in the H2D stream, and what follows the last
H2D (the tail: last fold + D2H).

    python scripts/e2e_timeline.py DIR
"""
import csv
import glob
import os
import statistics
import sys


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    copies = load(d, "*memory_copy_trace.csv")
    kernels = load(d, "*kernel_trace.csv")
    ev = []
    for r in copies:
        kind = r.get("Direction") or r.get("Operation") or ""
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "D2H" if "DEVICE_TO_HOST" in kind else
                   "H2D" if "HOST_TO_DEVICE" in kind else kind, int(r.get("Bytes", 0) or 0)))
    for r in kernels:
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"][:30], 0))
    ev.sort()
    rounds, cur = [], [ev[0]]
    for e in ev[1:]:
        if e[0] - max(x[1] for x in cur) > 1_000_000:
            rounds.append(cur)
            cur = []
        cur.append(e)
    rounds.append(cur)
    big = [r for r in rounds if sum(x[3] for x in r if x[2] == "H2D") > 100e6]
    print(f"# {d}\n\n{len(big)} rounds with > 100 MB of H2D\n")
    print("| round | span ms | H2D bytes | H2D busy ms | H2D GB/s while busy | H2D gaps ms | tail after last H2D ms |")
    print("|---|---|---|---|---|---|---|")
    for i, r in enumerate(big):
        h2d = sorted(x for x in r if x[2] == "H2D")
        t0, t1 = r[0][0], max(x[1] for x in r)
        busy, gaps, end = 0, 0, h2d[0][0]
        for s, e, _, _ in h2d:
            if s > end:
                gaps += s - end
            busy += e - max(s, end) if e > end else 0
            end = max(end, e)
        nbytes = sum(x[3] for x in h2d)
        print(f"| {i} | {(t1 - t0) / 1e6:.2f} | {nbytes / 1e6:.0f} MB | {busy / 1e6:.2f} | "
              f"{nbytes / busy / 1e3 if busy else 0:.1f} | {gaps / 1e6:.2f} | {(t1 - end) / 1e6:.2f} |")


if __name__ == "__main__":
    main()
