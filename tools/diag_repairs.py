"""Relaxation repairs on the sparse-failure regime of test_sparse_boundary_failures
(true tuning, short warm-up) for a few segment grids: how many chunks each E-step
recomputes against the number of chunks.  A metric that cannot resolve the tolerance
makes every failure cascade to its segment's end (repairs ~ chunks / 2 at 4 segments).

usage: python tools/diag_repairs.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from synth import make
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, ScanConfig
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    N, L, T = 256, 128, 8000
    d = make(N, L, T)
    sp = SpikeData(d['y'])
    for chunk, warm, seg in ((8, 2, 0), (8, 2, 4), (8, 4, 4), (16, 8, 4), (32, 16, 4)):
        eng = DeviceEM(sp, L, basis=d['B'], scan=ScanConfig(chunk=chunk, warmup=warm, relax_segments=seg))
        eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
        eng.set_tuning(d['tuning'])
        logz = torch.zeros(1, dtype=torch.float64, device='cuda')
        eng.e_step(1.0, logz)
        f, b = eng.repairs()
        rf, rb = eng.relax_rounds()
        print(json.dumps({"chunk": chunk, "warmup": warm, "segments": seg, "chunks": -(-T // chunk),
                          "repairs": [f, b], "rounds": [rf, rb]}), flush=True)


if __name__ == "__main__":
    main()
