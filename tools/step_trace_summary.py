"""Summarise a rocprofv3 kernel trace of one-launch steps (scripts/step_trace.sh):
for each fold launch, when each round's waiter returned and when the kernels
queued behind the waiters (the round's exchange) started and ended, relative
to the fold launch's start and end (microseconds)."""
import csv
import sys


def main(path: str) -> None:
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["t0"])
    folds = [r for r in rows if "_step<" in r["Kernel_Name"]]
    waits = [r for r in rows if "k_wait_round" in r["Kernel_Name"]]
    print(f"{path}: {len(folds)} step launches, {len(waits)} round waits")
    for f in folds[-5:]:
        dur = (f["t1"] - f["t0"]) / 1e3
        ws = [w for w in waits if f["t0"] <= w["t1"] <= f["t1"] + 200_000]  # returned during this launch
        ends = [(w["t1"] - f["t0"]) / 1e3 for w in ws]
        after = [r for r in rows if r is not f and r["Queue_Id"] != f["Queue_Id"] and "k_wait_round" not in r["Kernel_Name"]
                 and f["t0"] < r["t0"] < f["t1"] + 200_000]
        ex = [(r["Kernel_Name"].split("(")[0][-40:], round((r["t0"] - f["t0"]) / 1e3, 1), round((r["t1"] - f["t0"]) / 1e3, 1))
              for r in after[:8]]
        print(f"  fold {dur:8.1f} us; round waits returned at {[round(e, 1) for e in ends]} us after its start; "
              f"other queues' kernels (start, end): {ex}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
