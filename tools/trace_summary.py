"""Per-kernel mean duration over the TIMED dispatches of a bench run under
`rocprofv3 --kernel-trace` (the last `steps` EM iterations' launches of each kernel),
for comparison with bench.py's live HIP-event timings (its `rooflines[*].ms` and
`kernels_ms`).  `iters` = every EM iteration the run executed (bench.py: 1 pre-warm +
2 x (warmup + steps): the measured fit and the instrumented one, e.g. 51 for --warmup 5
--steps 20), so a kernel launched k times per iteration keeps its last k*steps.  Per-fit
kernels (spike preparation, the first M-step's exp) are listed with their own counts.
usage: python tools/trace_summary.py gpurun_out/prof_X/run_kernel_trace.csv STEPS ITERS out.csv
"""
import csv
import sys
from collections import defaultdict


def main(path, steps, iters, out):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows = []
    for k, v in d.items():
        v.sort()
        per_iter = max(1, len(v) // iters)
        last = v[-steps * per_iter:]
        us = [(e - s) / 1e3 for s, e in last]
        rows.append((k, len(v), len(last), sum(us) / len(us), sum(us) / steps))
    rows.sort(key=lambda x: -x[4])
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "dispatches_total", "dispatches_timed", "mean_us_timed", "us_per_em_iteration"])
        for r in rows:
            w.writerow([r[0], r[1], r[2], round(r[3], 2), round(r[4], 2)])
    for r in rows[:14]:
        print(f"{r[0][:60]:60s} {r[3]:9.2f} us/launch {r[4]:9.2f} us/iter ({r[2]} timed of {r[1]})")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
