#!/usr/bin/env python3
"""Per-round DMA timeline of an end-to-end run (rocprofv3 --kernel-trace
--memory-copy-trace of bench_e2e.py).  Rounds are the runs of host-to-device
copies separated by more than 250 us of idle copy engine; per round: the
number of DMAs, their durations (the chunk ramps show up here), the copy
engine's busy time and its idle gaps inside the round, and the idle time
between rounds (the previous round's tail + this round's head).

    python scripts/e2e_timeline.py DIR
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
    h = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "HOST_TO_DEVICE" in r["Direction"]]
    segs, cur = [], [h[0]]
    between = []
    for a, b in zip(h, h[1:]):
        if b[0] - a[1] > 250_000:
            segs.append(cur)
            between.append(b[0] - a[1])
            cur = []
        cur.append(b)
    segs.append(cur)
    print(f"# {d}\n")
    print("| round | DMAs | span us | DMA busy us | idle inside us | idle before the round us | DMA durations us |")
    print("|---|---|---|---|---|---|---|")
    for i, s in enumerate(segs):
        busy = sum(e - b for b, e in s)
        inside = sum(max(0, s[j + 1][0] - s[j][1]) for j in range(len(s) - 1))
        before = between[i - 1] / 1e3 if i > 0 else float("nan")
        durs = " ".join(str(round((e - b) / 1e3)) for b, e in s)
        print(f"| {i} | {len(s)} | {(s[-1][1] - s[0][0]) / 1e3:.0f} | {busy / 1e3:.0f} | {inside / 1e3:.0f} | "
              f"{before:.0f} | {durs} |")


if __name__ == "__main__":
    main()
