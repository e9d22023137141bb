"""Host-side timeline of the public fit_em(n_iter=20) at C3, cold (first public fit of the
process) and warm: when the y upload / spike preparation, the posterior-init upload, each
page-locked result buffer's allocation (helper thread), the enqueue of the EM loop and the
final synchronisation start and end, in ms from the call.  Run on the GPU box:
python tools/api_fit_phases.py > gpurun_out/api_fit_phases.json"""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth  # noqa: E402


def main():
    N, T, L = 512, 100000, 512
    y, B, W0, lp0 = synth(N, T, L)
    import poor_man_gplvm_amd.core as core
    from poor_man_gplvm_amd import PoissonGPLVMJump1D
    from poor_man_gplvm_amd import _native as nat
    ev = []
    t0 = [0.0]
    lock = threading.Lock()

    def rec(name, a, b):
        with lock:
            ev.append((name, round((a - t0[0]) * 1e3, 2), round((b - t0[0]) * 1e3, 2),
                       threading.current_thread().name[:12]))

    def wrap(obj, attr, name):
        fn = getattr(obj, attr)

        def w(*a, **k):
            s = time.perf_counter()
            r = fn(*a, **k)
            rec(name, s, time.perf_counter())
            return r
        setattr(obj, attr, w)

    wrap(nat, 'host_array', 'host_array')
    wrap(core, 'SpikeData', 'SpikeData')
    wrap(core.DeviceEM, 'set_log_posterior', 'set_log_posterior')
    wrap(core.DeviceEM, 'm_step', 'm_step_enqueue')
    wrap(core.DeviceEM, 'e_step', 'e_step_enqueue')
    wrap(core._PinnedCopies, 'finish', 'finish')
    wrap(core._PinnedCopies, 'submit', 'submit')
    m = PoissonGPLVMJump1D(N, n_latent_bin=L, tuning_lengthscale=10.0)
    m.tuning_basis, m.params = B, W0
    if '--engine-prewarm' in sys.argv:
        # as bench.py: only the engine's own kernels have run before the public fit
        from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig
        from poor_man_gplvm_amd.gp_kernel import banded_transition
        eng = DeviceEM(SpikeData(y), L, basis=B)
        eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
        eng.set_log_posterior(lp0)
        dev = eng.dev
        W = torch.as_tensor(W0.astype(np.float64), device=dev)
        mu, nu = torch.zeros_like(W), torch.zeros_like(W)
        cnt = torch.zeros(1, dtype=torch.int64, device=dev)
        st = torch.zeros(4, dtype=torch.float64, device=dev)
        lh = torch.zeros(1000, dtype=torch.float64, device=dev)
        eh = torch.zeros_like(lh)
        lz = torch.zeros(1, dtype=torch.float64, device=dev)
        for _ in range(3):
            eng.m_step(W, mu, nu, cnt, AdamConfig(), st, lh, eh)
            eng.compute_tuning(W)
            eng.e_step(1.0, lz)
        torch.cuda.synchronize()
    else:
        m.fit_em(y[:2000], n_iter=2, log_posterior_init=lp0[:2000])           # code objects
    out = {'thp': open('/sys/kernel/mm/transparent_hugepage/enabled').read().strip()
           if os.path.exists('/sys/kernel/mm/transparent_hugepage/enabled') else None,
           'thp_defrag': open('/sys/kernel/mm/transparent_hugepage/defrag').read().strip()
           if os.path.exists('/sys/kernel/mm/transparent_hugepage/defrag') else None}
    for run in ('cold', 'warm'):
        ev.clear()
        m.params = W0
        torch.cuda.synchronize()
        t0[0] = time.perf_counter()
        res = m.fit_em(y, n_iter=20, log_posterior_init=lp0)
        torch.cuda.synchronize()
        total = round((time.perf_counter() - t0[0]) * 1e3, 2)
        out[run] = {'total_ms': total, 'events': sorted(ev, key=lambda e: e[1])}
        del res
        import gc
        gc.collect()
    print(json.dumps(out))


if __name__ == '__main__':
    main()
