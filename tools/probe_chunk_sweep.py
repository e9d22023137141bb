"""Diagnostic (not collected): the C3 scan main passes at several chunk lengths.

After n EM iterations of a C3 fit, times the forward main pass (phase 1) with and without
its alpha stores, and the backward main pass, at chunk lengths C (M = T / C chains, one
wave each), so the cost of the alpha write stream can be compared at 2 and 4 waves per
SIMD (C = 49 / 25) -- the question behind splitting one chain over several waves."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.probe_scan_phases import timed  # noqa: E402


def main():
    import torch
    from bench import synth, CONFIGS
    from poor_man_gplvm_amd import _native as nat
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    n_it = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    N, T, L = CONFIGS['c3']
    y, B, W0, lp0 = synth(N, T, L)
    dev = torch.device('cuda', 0)
    eng = DeviceEM(SpikeData(y), L, basis=B, scan=ScanConfig())
    eng.adaptive = True
    eng.set_transition(banded_transition(L, 1.0, 0.01, 0.01))
    eng.set_log_posterior(lp0)
    lib = eng.lib
    W = torch.as_tensor(W0.astype(np.float64), device=dev).contiguous()
    mu, nu = torch.zeros_like(W), torch.zeros_like(W)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.zeros(4, dtype=torch.float64, device=dev)
    lh = torch.zeros(1000, dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    lz = torch.zeros(1, dtype=torch.float64, device=dev)
    for it in range(n_it):
        eng.m_step(W, mu, nu, cnt, AdamConfig(), st, lh, eh)
        eng.compute_tuning(W)
        eng.e_step(1.0, lz)
    torch.cuda.synchronize()
    res = {'n_it': n_it, 'C_default': eng.C, 'Cb_default': eng.Cb}
    ws = torch.zeros(int(lib.pmg_fwdbwd_workspace_size(T, L, 16)), dtype=torch.uint8, device=dev)

    def fwd(C, Wm, bits):
        args = (nat.ptr(eng.delta), nat.ptr(eng.phi), nat.ptr(eng.mref), T, ctypes.byref(eng._tr_c), 1.0, C, Wm,
                float(eng.scan.tol), nat.ptr(eng.alpha), nat.ptr(eng.logc), nat.ptr(lz), nat.ptr(ws),
                ws.numel(), nat.stream_handle())
        return lambda: nat.check(lib.pmg_forward_filter_phase(*args, 1 | bits), "fwd")

    def bwd(C, Wm):
        args = (nat.ptr(eng.delta), nat.ptr(eng.phi), nat.ptr(eng.alpha), T, ctypes.byref(eng._tr_c), 1.0, C, Wm,
                float(eng.scan.tol), nat.ptr(eng._P), None, None, nat.ptr(ws), ws.numel(),
                nat.stream_handle())
        return lambda: nat.check(lib.pmg_backward_smoother_phase(*args, 1), "bwd")

    for C in (25, 33, 49, 65, 98):
        for Wm in (0, 48):
            res[f'fwd_c{C}_w{Wm}_us'] = round(1e3 * timed(fwd(C, Wm, nat.PHASE_NO_JUMP_ROWS)), 1)
            res[f'fwd_noalpha_c{C}_w{Wm}_us'] = round(1e3 * timed(fwd(C, Wm, nat.PHASE_NO_ALPHA)), 1)
        print(json.dumps(res), flush=True)
    fwd(eng.C, 48, nat.PHASE_NO_JUMP_ROWS)()
    for C in (49, 65, 98, 196):
        for Wm in (0, 48):
            res[f'bwd_c{C}_w{Wm}_us'] = round(1e3 * timed(bwd(C, Wm)), 1)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
