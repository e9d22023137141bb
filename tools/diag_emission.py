"""Time the Poisson emission kernels at a BASELINE shape (default C3: N=512, L=512,
T=1e5): k_emission_i8 (PMG_EMISSION_PIPE=0, MT=1/2) against the pipelined
k_emission_pipe (PMG_EMISSION_PIPE=1), each call = k_rates_prepare + the GEMM kernel,
back to back on the engine's stream; checks the outputs are bit-identical.

usage: python tools/diag_emission.py [--T 100000] [--N 512] [--L 512] [--reps 30]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=100000)
    ap.add_argument("--N", type=int, default=512)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma list of variants (i8_mt1, i8_mt2, pipe)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from poor_man_gplvm_amd.engine import DeviceEM, SpikeData
    rng = np.random.default_rng(0)
    y = rng.poisson(0.3, size=(a.T, a.N)).astype(np.float32)
    tun = rng.uniform(0.01, 2.0, size=(a.L, a.N))
    eng = DeviceEM(SpikeData(y), a.L)
    eng.set_tuning(tun)
    res, outs = {}, {}
    variants = [v for v in (("i8_mt1", "0", "1"), ("i8_mt2", "0", "2"), ("pipe", "1", "1"), ("yreg", "auto", "1"))
                if not a.only or v[0] in a.only.split(",")]
    for name, pipe, mt in variants:
        os.environ["PMG_EMISSION_PIPE"], os.environ["PMG_EMISSION_MT"] = pipe, mt
        for _ in range(1 if a.reps <= 2 else 3):
            eng.emission(1.0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            eng.emission(1.0)
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t) / a.reps * 1e6
        eng.emission_status()
        outs[name] = (eng.delta.cpu().numpy().copy(), eng.rblk.cpu().numpy().copy())
    ref = outs[variants[0][0]]
    same = {k: bool(all(np.array_equal(x, y) for x, y in zip(ref, v))) for k, v in outs.items()}
    line = {"shape": {"T": a.T, "N": a.N, "L": a.L}, "us_per_call": {k: round(v, 1) for k, v in res.items()},
            "bit_identical_to_first": same}
    print(json.dumps(line))
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
