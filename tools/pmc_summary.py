"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) into profiles/<out>.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KB).  The factor
2 is the gfx950 correction of MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts
128-B memory-side read requests as 64 B for wide coalesced streaming reads.
Only the last LAST_ITERS EM iterations' dispatches of each kernel count (steady state:
the first iterations of a fresh fit run long relaxations and Adam loops).
usage: python tools/pmc_summary.py gpurun_out/pmc1 profiles/r02_pmc_c3.json [ITERS LAST_ITERS]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

KEYS = {"k_forward<": "k_forward", "k_backward<": "k_backward", "k_ptb3": "k_ptb3",
        "k_emission_i8": "k_emission_i8", "k_emission_yreg": "k_emission_yreg",
        "k_emission_pipe": "k_emission_pipe", "k_adam<": "k_adam", "k_verify": "k_verify",
        "k_forward_relax<": "k_forward_relax", "k_backward_relax<": "k_backward_relax"}


def main(prefix, out, iters=7, last_iters=3):
    vals = defaultdict(lambda: defaultdict(list))
    for tag in ("fetch", "write", "sq", "sq2"):
        files = glob.glob(f"{prefix}_{tag}/**/*counter_collection.csv", recursive=True)
        per = defaultdict(lambda: defaultdict(list))     # kernel -> counter -> [(dispatch, value)]
        for f in files:
            for r in csv.DictReader(open(f)):
                for pat, k in KEYS.items():
                    if pat in r["Kernel_Name"]:
                        per[k][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for k, cs in per.items():
            for c, dv in cs.items():
                dv.sort()
                keep = max(1, len(dv) // iters) * last_iters
                vals[k][c].extend(v for _, v in dv[-keep:])
    res = {}
    for k, cs in vals.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"counters_mean_per_dispatch": mean, "dispatches": max(len(v) for v in cs.values())}
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            e["hbm_read_bytes_per_launch"] = 2.0 * mean["FETCH_SIZE"] * 1024.0
            e["hbm_write_bytes_per_launch"] = mean["WRITE_SIZE"] * 1024.0
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
        res[k] = e
    doc = {"source": f"rocprofv3 --pmc passes, {prefix}_*, bench.py --steps 3 --warmup 3 (+1 pre-warm iteration); "
                     f"means over the last {last_iters} of {iters} EM iterations' dispatches",
           "note": "FETCH_SIZE doubled (gfx950 correction); values are means over the profiled dispatches",
           "kernels": res}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, e in res.items():
        print(k, {x: round(e[x] / 1e6, 1) for x in e if x.endswith("per_launch")})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:5]))
