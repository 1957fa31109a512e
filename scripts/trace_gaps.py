#!/usr/bin/env python3
"""From a rocprofv3 kernel trace (CSV) of a bench.py run with rounds: the GPU
timeline over the timed steps (the last STEPS x ROUNDS fold dispatches): per
kernel kind the count, mean duration and hardware queue, the gap from one
fold's end to the next fold's start, and how many exchange kernels ran
concurrently with a fold.

    python scripts/trace_gaps.py DIR [DIR ...]     (env STEPS, default 30)
"""
import csv
import glob
import os
import statistics
import sys

KINDS = ("k_fedavg_bf16", "k_fold_f32", "k_read_sweep", "k_synth", "nccl", "copyBuffer", "fillBuffer",
         "FillFunctor")


def kind(name):
    for k in KINDS:
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main():
    steps = int(os.environ.get("STEPS", "30"))
    for d in sys.argv[1:]:
        f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if not f:
            print(f"## {d}\n\nno kernel trace\n")
            continue
        rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
        ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"]), r.get("Queue_Id"))
              for r in rows]
        folds = [i for i, e in enumerate(ev) if e[2] in ("k_fedavg_bf16", "k_fold_f32")]
        rounds = int(os.environ.get("ROUNDS", "0")) or None
        n_timed = steps * rounds if rounds else len(folds) // 2
        win = folds[-n_timed:]
        t0, t1 = ev[win[0]][0], ev[win[-1]][1]
        inwin = [e for e in ev if e[0] >= t0 and e[1] <= t1]
        gaps = [ev[b][0] - ev[a][1] for a, b in zip(win, win[1:])]
        fold_iv = [(ev[i][0], ev[i][1]) for i in win]
        others = [e for e in inwin if e[2] not in ("k_fedavg_bf16", "k_fold_f32")]
        overl = sum(1 for s, e, _, _ in others if any(fs < e and s < fe for fs, fe in fold_iv))
        busy = sum(ev[i][1] - ev[i][0] for i in win)
        print(f"## {os.path.basename(d.rstrip('/'))}\n")
        print(f"timed window {(t1 - t0) / 1e3:.1f} us over {len(win)} folds: folds busy {busy / (t1 - t0):.3f}; "
              f"fold-to-fold gap median {statistics.median(gaps) / 1e3:.1f} us, mean {statistics.mean(gaps) / 1e3:.1f} us; "
              f"{overl} of {len(others)} other kernels overlapped a fold\n")
        print("| kernel | count | mean us | hardware queues |")
        print("|---|---|---|---|")
        by = {}
        for s, e, k, q in inwin:
            by.setdefault(k, []).append((e - s, q))
        for k, v in sorted(by.items(), key=lambda kv: -sum(x for x, _ in kv[1])):
            print(f"| `{k}` | {len(v)} | {statistics.mean(x for x, _ in v) / 1e3:.1f} | "
                  f"{', '.join(sorted({str(q) for _, q in v}))} |")
        print()


if __name__ == "__main__":
    main()
