"""Boundary-distance diagnostics for the time-parallel scan (repairs disabled)."""
import os, sys
os.environ["PMG_DEBUG_NO_REPAIR"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import bench
from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, ScanConfig
from poor_man_gplvm_amd.gp_kernel import banded_transition

def carve(ws, T, Lpad, C):
    M = (T + C - 1) // C
    off = 0
    out = {}
    def take(name, n, dt):
        nonlocal off
        off = (off + 255) & ~255
        nbytes = n * np.dtype(dt).itemsize
        out[name] = ws[off:off + nbytes].view(dt)
        off += nbytes
    take('repairs', 64, np.int32)
    take('jsc', 2 * T, np.float32)
    for k in ['s_in', 's_out', 'b_in', 'b_first']:
        take(k, M * 2 * Lpad, np.float32)
    return out, M

def hil(x, y, lo=1e-30):
    x = x.astype(np.float64) / x.max(); y = y.astype(np.float64) / y.max()
    m = (x > lo) & (y > lo)
    r = np.log(x[m]) - np.log(y[m])
    bad = np.any((np.maximum(x, y) > 1e-20) & ~m)
    return (r.max() - r.min()) if m.any() else 0.0, bad

def run(cfg, warms, chunk=0, iters_model=True):
    N, T, L = bench.CONFIGS[cfg]
    y, B, W0, lp0 = bench.synth(N, T, L)
    from oracle import gplvm_oracle as O
    W = np.random.default_rng(0).normal(size=(B.shape[1], N))  # true W
    tun = np.logaddexp(B.astype(np.float64) @ W, 0.0)
    sp = SpikeData(y)
    Lpad = 64 * next(j for j in (1, 2, 4, 8, 16) if L <= 64 * j)
    for tname, tuning in [('true', tun), ('random', np.logaddexp(B.astype(np.float64) @ W0.astype(np.float64), 0.0))]:
        for w in warms:
            eng = DeviceEM(sp, L, basis=B, scan=ScanConfig(chunk=chunk or None, warmup=w, adaptive=False))
            eng.set_transition(banded_transition(L, 1.0))
            eng.set_tuning(tuning)
            eng.emission(1.0)
            lz = torch.zeros(1, dtype=torch.float64, device='cuda')
            eng.forward(1.0, lz)
            eng.backward(1.0, True)
            torch.cuda.synchronize()
            ws = eng.ws_fb.cpu().numpy()
            a, M = carve(ws, T, Lpad, eng.C)
            sh = (M, 2 * Lpad)
            si, so, bi, bo = [a[k].reshape(sh) for k in ['s_in', 's_out', 'b_in', 'b_first']]
            fd = [hil(si[c], so[c - 1]) for c in range(1, M)]
            bd = [hil(bi[c], bo[c + 1]) for c in range(0, M - 1)]
            fdv = np.array([d for d, _ in fd]); bdv = np.array([d for d, _ in bd])
            print(f"{cfg} tuning={tname} C={eng.C} warm={w}: fwd d: med {np.median(fdv):.2e} p99 {np.quantile(fdv,.99):.2e} max {fdv.max():.2e} bad {sum(b for _,b in fd)} | "
                  f"bwd d: med {np.median(bdv):.2e} p99 {np.quantile(bdv,.99):.2e} max {bdv.max():.2e} bad {sum(b for _,b in bd)}", flush=True)
            # restricted metric: components > 1e-10
            fd2 = np.array([hil(si[c], so[c - 1], 1e-10)[0] for c in range(1, M)])
            bd2 = np.array([hil(bi[c], bo[c + 1], 1e-10)[0] for c in range(0, M - 1)])
            print(f"      (>1e-10) fwd max {fd2.max():.2e} p99 {np.quantile(fd2,.99):.2e} | bwd max {bd2.max():.2e} p99 {np.quantile(bd2,.99):.2e}", flush=True)

if __name__ == '__main__':
    torch.cuda.set_device(0)
    run('c1', [48, 128])
    run('c2', [48])
    run('c3', [32, 64])
