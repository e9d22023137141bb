"""Where the wall time of the public fit_em(n_iter=20) at C3 goes (host side): upload and
prepare of y, the device EM loop, and each returned array's device->host copy / host op.
Run on the GPU box: python tools/api_fit_profile.py > gpurun_out/api_fit_profile.json"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth  # noqa: E402


def main():
    N, T, L = 512, 100000, 512
    y, B, W0, lp0 = synth(N, T, L)
    from poor_man_gplvm_amd import PoissonGPLVMJump1D
    from poor_man_gplvm_amd.engine import SpikeData
    out = {}

    def tick(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        out[name] = round(time.perf_counter() - t0, 5)
        return r
    m = PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.0)
    m.tuning_basis, m.params = B, W0
    m.fit_em(y[:2000], n_iter=2, log_posterior_init=lp0[:2000])           # code objects
    tick('spikes_upload_prepare', lambda: SpikeData(y))
    g = torch.rand((T, 2, L), device='cuda')
    tick('d2h_pageable_T2L', lambda: g.cpu().numpy())
    pin = torch.empty((T, 2, L), dtype=torch.float32, pin_memory=True)
    tick('pinned_alloc_T2L', lambda: torch.empty((T, 2, L), dtype=torch.float32, pin_memory=True))
    tick('d2h_pinned_T2L', lambda: pin.copy_(g))
    h = g.cpu().numpy()
    tick('host_sum_axis1', lambda: h.sum(axis=1))
    tick('host_sum_axis2', lambda: h.sum(axis=2))
    tick('device_log', lambda: torch.log(g))
    tick('fit_em_api_20', lambda: m.fit_em(y, n_iter=20, log_posterior_init=lp0))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
