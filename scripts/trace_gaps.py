#!/usr/bin/env python3
"""From a rocprofv3 kernel trace (CSV), the GPU timeline of the last timed
steps: per kernel name the count and mean duration, the busy fraction of the
span covered by kernels, and the idle gaps between consecutive kernels.

    python scripts/trace_gaps.py DIR [DIR ...]
"""
import csv
import glob
import os
import statistics
import sys


def main():
    for d in sys.argv[1:]:
        f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if not f:
            print(f"{d}: no kernel trace")
            continue
        rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
        # the timed region: the last 60 % of the kernels (after input generation and warmup)
        rows = rows[int(len(rows) * 0.4):]
        spans = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
        t0, t1 = spans[0][0], max(e for _, e, _ in spans)
        busy, cur_s, cur_e = 0, spans[0][0], spans[0][1]
        gaps = []
        for s, e, _ in spans[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        by = {}
        for s, e, n in spans:
            short = n.split("(")[0][-60:]
            by.setdefault(short, []).append(e - s)
        print(f"## {d}\n")
        print(f"span {(t1 - t0) / 1e6:.3f} ms, kernels busy {busy / (t1 - t0):.3f}, "
              f"{len(gaps)} gaps, mean {statistics.mean(gaps) / 1e3 if gaps else 0:.1f} us, "
              f"total {sum(gaps) / 1e6:.3f} ms\n")
        print("| kernel | count | mean us |")
        print("|---|---|---|")
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f"| `{k}` | {len(v)} | {statistics.mean(v) / 1e3:.1f} |")
        print()


if __name__ == "__main__":
    main()
