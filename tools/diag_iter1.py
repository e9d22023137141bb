"""Per-iteration breakdown of the first EM iterations of a fresh C3 fit (the bench's
fresh_fit.warmup_iteration_s): section times (KernelTimer), relaxation repairs / rounds
and wall time per iteration, for a few scan warm-up settings.

usage: python tools/diag_iter1.py [--config c3] [--iters 4] [--warms 48,128] [--out f.json]
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
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--warms", default="48,128")
    ap.add_argument("--out", default=None)
    ap.add_argument("--segs", default="0", help="relaxation segments per sequence, comma list (0: library default)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig, KernelTimer
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    N, T, L = bench.CONFIGS[a.config]
    y, B, W0, lp0 = bench.synth(N, T, L, rank=0)
    dev = torch.device("cuda", 0)
    adam = AdamConfig(lr=0.01, maxiter=1000, tol=1e-6, prior_std=1.0)
    lines = []
    for warm, segs in [(int(w), int(sg)) for w in a.warms.split(",") for sg in a.segs.split(",")]:
        eng = DeviceEM(SpikeData(y), L, basis=B, scan=ScanConfig(warmup=warm, relax_segments=segs))
        eng.adaptive = True
        eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
        W = torch.empty((B.shape[1], N), dtype=torch.float64, device=dev)
        mu, nu = torch.zeros_like(W), torch.zeros_like(W)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        stats = torch.zeros((a.iters, 4), dtype=torch.float64, device=dev)
        lh = torch.zeros((a.iters, adam.maxiter), dtype=torch.float64, device=dev)
        eh = torch.zeros_like(lh)
        logz = torch.zeros(a.iters, dtype=torch.float64, device=dev)
        for rep in range(2):   # rep 0 pre-warms the code objects
            eng.set_log_posterior(lp0)
            eng.reset_adaptive()
            W.copy_(torch.as_tensor(W0.astype(np.float64), device=dev))
            mu.zero_()
            nu.zero_()
            cnt.zero_()
            eng.warm = [warm, warm]
            for i in range(a.iters):
                timer = KernelTimer()
                eng.timer = timer if rep else None
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.m_step(W, mu, nu, cnt, adam, stats[i], lh[i], eh[i])
                eng.compute_tuning(W)
                eng.e_step(1.0, logz[i:i + 1])
                torch.cuda.synchronize()
                wall = time.perf_counter() - t0
                eng.timer = None
                if rep:
                    s = timer.summary()
                    line = {"warm": warm, "segs": segs, "iter": i + 1, "wall_ms": round(1e3 * wall, 3),
                            "sections_ms": {k: round(v[1], 4) for k, v in s.items()},
                            "repairs": list(eng.repairs()), "relax_rounds": list(eng.relax_rounds()),
                            "adam_iters": float(stats[i, 0].item()), "logz": float(logz[i].item())}
                    print(json.dumps(line), flush=True)
                    lines.append(line)
        del eng
        torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as f:
            for line in lines:
                f.write(json.dumps(line) + "\n")


if __name__ == "__main__":
    main()
