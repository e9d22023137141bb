"""Per-kernel mean duration over the TIMED dispatches of a bench run under
`rocprofv3 --kernel-trace` (the last `steps` launches of each kernel), for comparison
with bench.py's live HIP-event timings (its `rooflines[*].ms`).
usage: python tools/trace_summary.py gpurun_out/prof_X/run_kernel_trace.csv STEPS out.csv
"""
import csv
import sys
from collections import defaultdict


def main(path, steps, out):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows = []
    for k, v in d.items():
        v.sort()
        per_step = max(1, len(v) // 13) if len(v) >= 13 else 1
        last = v[-steps * per_step:]
        us = [(e - s) / 1e3 for s, e in last]
        rows.append((k, len(v), len(last), sum(us) / len(us)))
    rows.sort(key=lambda x: -x[3] * x[2])
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "dispatches_total", "dispatches_timed", "mean_us_timed"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 2)])
    for r in rows[:10]:
        print(f"{r[0][:60]:60s} {r[3]:10.2f} us  ({r[2]} timed of {r[1]})")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
