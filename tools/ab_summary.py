"""Summarise tools/gpu_bench_ab.sh outputs: value and per-section kernel ms per run."""
import glob
import json
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable", e)
        continue
    k = d.get("kernels_ms", {})
    ks = " ".join(f"{n}={v:.4f}" for n, v in sorted(k.items()) if isinstance(v, (int, float)))
    print(f"{f.split('/')[-1]:28s} {d['value']:8.1f} frac={d['roofline']['frac']:.3f}  {ks}")
