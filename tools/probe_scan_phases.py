"""Diagnostic (not collected): where the C3 scan main passes spend their time.

After n EM iterations of a C3 fit, times the forward / backward MAIN passes alone (phase 1)
for several warm-ups, with and without the forward's alpha stores (PMG_PHASE_NO_ALPHA), and
measures the chip's streaming read / copy / triad bandwidth on buffers of the scan's size,
so the output steps (read delta + write alpha, or read delta + alpha + write P) can be
priced against the mixed read/write rate the HBM actually sustains."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps=20):
    import torch
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


def bandwidth(out):
    import torch
    n = 100_000 * 512
    x = torch.rand(n, device='cuda')
    y = torch.rand(n, device='cuda')
    z = torch.empty(n, device='cuda')
    B = 4 * n
    r = timed(lambda: torch.sum(x))
    out['bw_read_TBs'] = B / r / 1e9
    c = timed(lambda: z.copy_(x))
    out['bw_copy_TBs'] = 2 * B / c / 1e9
    t = timed(lambda: torch.add(x, y, out=z))
    out['bw_triad_TBs'] = 3 * B / t / 1e9
    w = timed(lambda: z.fill_(1.0))
    out['bw_write_TBs'] = B / w / 1e9


def main():
    import torch
    from bench import synth, CONFIGS
    from poor_man_gplvm_amd import _native as nat
    from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig
    from poor_man_gplvm_amd.gp_kernel import banded_transition
    n_it = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    quick = len(sys.argv) > 2 and sys.argv[2] == 'quick'
    res = {'n_it': n_it, 'lib': os.environ.get('PMG_LIB_PATH', 'tree')}
    if not quick:
        bandwidth(res)
        print(json.dumps(res), flush=True)
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
    adam = AdamConfig()
    st = torch.zeros(4, dtype=torch.float64, device=dev)
    lh = torch.zeros(1000, dtype=torch.float64, device=dev)
    eh = torch.zeros_like(lh)
    lz = torch.zeros(1, dtype=torch.float64, device=dev)
    for it in range(n_it):
        eng.m_step(W, mu, nu, cnt, adam, st, lh, eh)
        eng.compute_tuning(W)
        eng.e_step(1.0, lz)
    torch.cuda.synchronize()
    C, Cb = eng.C, eng.Cb
    res['C'], res['Cb'] = C, Cb

    def fwd(Wm, bits):
        args = (nat.ptr(eng.delta), nat.ptr(eng.phi), nat.ptr(eng.mref), T, ctypes.byref(eng._tr_c), 1.0, C, Wm,
                float(eng.scan.tol), nat.ptr(eng.alpha), nat.ptr(eng.logc), nat.ptr(lz), nat.ptr(eng.ws_fb),
                eng.ws_fb.numel(), nat.stream_handle())
        return lambda: nat.check(lib.pmg_forward_filter_phase(*args, 1 | bits), "fwd")

    def bwd(Wm):
        args = (nat.ptr(eng.delta), nat.ptr(eng.phi), nat.ptr(eng.alpha), T, ctypes.byref(eng._tr_c), 1.0, Cb, Wm,
                float(eng.scan.tol), nat.ptr(eng._P), None, None, nat.ptr(eng.ws_fb), eng.ws_fb.numel(),
                nat.stream_handle())
        return lambda: nat.check(lib.pmg_backward_smoother_phase(*args, 1), "bwd")

    for Wm in ((0, 48) if quick else (0, 8, 16, 32, 48, 96)):
        res[f'fwd_w{Wm}_us'] = 1e3 * timed(fwd(Wm, nat.PHASE_NO_JUMP_ROWS))
        res[f'fwd_noalpha_w{Wm}_us'] = 1e3 * timed(fwd(Wm, nat.PHASE_NO_ALPHA))
    # the forward again with alpha, so the backward reads a consistent alpha
    fwd(48, nat.PHASE_NO_JUMP_ROWS)()
    for Wm in ((0, 48) if quick else (0, 16, 48, 96)):
        res[f'bwd_w{Wm}_us'] = 1e3 * timed(bwd(Wm))
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
