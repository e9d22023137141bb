"""Mean duration of the C3 Poisson emission (digit preparation + k_emission_yreg + row
reference; N = L = 512, T = 1e5) over 50 calls (HIP events on the launch stream).  Run it
per library (PMG_LIB_PATH=exp/NAME/libpmg_hip.so for experiment variants)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from poor_man_gplvm_amd import _native as nat  # noqa: E402
from poor_man_gplvm_amd.engine import DeviceEM, SpikeData  # noqa: E402

N, T, L = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
y, B, W0, _ = bench.synth(N, T, L)
tun = np.logaddexp(B.astype(np.float64) @ W0.astype(np.float64), 0.0)
eng = DeviceEM(SpikeData(y), L, basis=B)
eng.set_tuning(tun)
for _ in range(5):
    eng.emission(1.0)
st = torch.cuda.current_stream()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(st)
for _ in range(50):
    eng.emission(1.0)
b.record(st)
b.synchronize()
print(os.environ.get("PMG_LIB_PATH", "tree"), "emission us per call", round(1e3 * a.elapsed_time(b) / 50, 1),
      "delta checksum", float(eng.delta.double().sum()), flush=True)
