#!/usr/bin/env python3
"""Parse a scripts/sweep_narrow2.sh log: per shape, auto vs the best variants."""
import re
import sys

txt = open(sys.argv[1]).read()
for block in txt.split("== ")[1:]:
    lines = block.strip().split("\n")
    res = []
    for ln in lines[1:]:
        m = re.match(r"variant (\d+) (\S+)\s+median ([\d.]+) ms\s+min ([\d.]+) ms\s+-> ([\d.]+) GB/s", ln)
        if m:
            res.append((float(m.group(3)), m.group(2), float(m.group(5))))
    res.sort()
    auto = [r for r in res if r[1] == "auto"]
    print(lines[0], "auto", auto[0][0] if auto else None, "ms",
          " | ".join(f"{n} {t:.4f} ms {g:.0f}" for t, n, g in res[:5]))
