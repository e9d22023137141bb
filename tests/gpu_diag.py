"""Component-by-component GPU vs oracle diagnostics (prints, does not assert)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from scipy.special import logsumexp
from oracle import gplvm_oracle as O
from tests.synth import make
import poor_man_gplvm_amd as P
from poor_man_gplvm_amd.engine import SpikeData, DeviceEM, AdamConfig, ScanConfig
from poor_man_gplvm_amd.gp_kernel import banded_transition

def rel(a, b, floor=1e-6):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / (np.abs(b) + floor)))

def run(N, L, T, chunk=None, warm=48, ls=10.0):
    print(f"=== N={N} L={L} T={T} chunk={chunk} warm={warm}", flush=True)
    d = make(N, L, T, ls=ls)
    y, B = d['y'], d['B']
    tun = d['tuning']
    sp = SpikeData(y)
    print("flags", sp.flags, "int_path", sp.int_path)
    eng = DeviceEM(sp, L, basis=B, scan=ScanConfig(chunk=chunk, warmup=warm))
    tr = banded_transition(L, 1.0)
    eng.set_transition(tr)
    eng.set_tuning(tun)
    # emission
    eng.emission(1.0)
    ll = eng.loglik().cpu().numpy()
    ll_ref = O.loglikelihood_poisson_all(y, tun)
    print("emission abs err", np.max(np.abs(ll - ll_ref)), "ref scale", np.abs(ll_ref).max())
    dref = ll_ref - ll_ref.max(1, keepdims=True)
    delta = eng.delta.cpu().numpy().astype(np.float64) + np.repeat(eng.rblk.cpu().numpy(), 32, axis=1)[:, :L] - eng.mref.cpu().numpy()[:, None]
    m = dref > -30
    print("emission rel-to-max err (within 30 nats)", np.max(np.abs(delta[m] - dref[m])))
    # f64 path
    sp64 = SpikeData(y); sp64.int_path = False
    e64 = DeviceEM(sp64, L, basis=B); e64.set_transition(tr); e64.set_tuning(tun); e64.emission(1.0)
    ll64 = e64.loglik().cpu().numpy()
    print("emission f64 path abs err", np.max(np.abs(ll64 - ll_ref)))
    # forward / backward
    logz = torch.zeros(1, dtype=torch.float64, device='cuda')
    gamma = torch.empty((T, 2, L), dtype=torch.float32, device='cuda')
    rho = torch.zeros((T, 2, L), dtype=torch.float32, device='cuda')
    torch.cuda.synchronize(); t0 = time.time()
    eng.forward(1.0, logz)
    eng.backward(1.0, True, gamma, rho)
    torch.cuda.synchronize(); print("fwd+bwd wall", time.time() - t0, "repairs", eng.repairs())
    K, logK, A, logA = O.create_transition_prob_1d(L, 1.0)
    t1 = time.time()
    out = O.smooth_all_step_combined_ma_chunk(y.astype(np.float64), tun, logK, logA, with_joint=(T * L * L <= 3e7))
    print("oracle time", time.time() - t1)
    lpa, lz, lca, cs, lj, _ = out
    post = np.exp(lpa)
    g = gamma.cpu().numpy()
    a = eng.alpha.cpu().numpy()
    print("logZ", float(logz.item()), lz, "rel", abs(logz.item() - lz) / abs(lz))
    print("logc max abs err", np.max(np.abs(eng.logc.cpu().numpy() - cs)))
    print("alpha (causal) max abs err", np.max(np.abs(a - np.exp(lca))))
    print("gamma max abs err", np.max(np.abs(g - post)), " rel(>1e-6)", rel(g[post > 1e-6], post[post > 1e-6], 0))
    plm = g.sum(1); plm_ref = post.sum(1)
    ok = np.abs(plm - plm_ref) <= 1e-5 * np.abs(plm_ref) + 1e-12
    print("posterior_latent_marg allclose(1e-5,1e-12) frac", ok.mean(), "max abs", np.max(np.abs(plm - plm_ref)))
    print("argmax match frac", np.mean(plm.argmax(1) == plm_ref.argmax(1)))
    P_ = eng.P.cpu().numpy()
    print("P vs gamma sum", np.max(np.abs(P_ - plm)))
    if lj is not None:
        S = eng.joint(rho).cpu().numpy()
        S4 = S.reshape(2, L, 2, L).transpose(0, 2, 1, 3)
        J = np.exp(logA)[:, :, None, None] * K[None] * S4
        print("joint max abs err", np.max(np.abs(J - np.exp(lj))), "sum", J.sum(), np.exp(lj).sum())
    # suff stats
    yw, tw = O.get_statistics(np.log(np.maximum(plm_ref, 1e-300)), y)
    eng.P.copy_(torch.as_tensor(plm_ref.astype(np.float32), device='cuda'))
    eng2 = eng
    lib = eng.lib
    from poor_man_gplvm_amd import _native as nat
    nat.check(lib.pmg_suffstats(nat.ptr(eng.P), nat.ptr(sp.yext), T, L, N, sp.Np, nat.ptr(eng.yw), nat.ptr(eng.tw), nat.ptr(eng.ws_ss), eng.ws_ss.numel(), nat.stream_handle()), 'ss')
    ywd = eng.yw.cpu().numpy(); twd = eng.tw.cpu().numpy()
    yw32, tw32 = O.get_statistics(np.log(np.maximum(plm_ref.astype(np.float32).astype(np.float64), 1e-300)), y)
    print("suffstats yw rel", rel(ywd, yw32, 1e-3), "tw rel", rel(twd, tw32, 1e-3))
    # adam fixed iterations
    for tol, mi in [(0.0, 30), (1e-6, 1000)]:
        Wd = torch.as_tensor(d['W0'].astype(np.float64), device='cuda').contiguous()
        mu = torch.zeros_like(Wd); nu = torch.zeros_like(Wd); cnt = torch.zeros(1, dtype=torch.int64, device='cuda')
        stats = torch.zeros(4, dtype=torch.float64, device='cuda'); lh = torch.zeros(mi, dtype=torch.float64, device='cuda'); eh = torch.zeros_like(lh)
        torch.cuda.synchronize(); t0 = time.time()
        eng.adam(Wd, mu, nu, cnt, AdamConfig(maxiter=mi, tol=tol), stats, lh, eh)
        torch.cuda.synchronize(); dt_ = time.time() - t0
        ref = O.adam_run(d['W0'].astype(np.float64), O.adam_init(d['W0']), 1.0, B.astype(np.float64), ywd, twd, maxiter=mi, tol=tol)
        s = stats.cpu().numpy()
        print(f"adam tol={tol}: n_iter {int(s[0])} vs {ref['n_iter']}  time {dt_*1e3:.2f} ms  W rel {rel(Wd.cpu().numpy(), ref['params'], 1e-3):.2e}  loss {s[1]} vs {ref['final_loss']}  err {s[2]} vs {ref['final_error']}  count {int(cnt.item())}")
        n = min(int(s[0]), ref['n_iter'])
        print("   loss hist rel", rel(lh.cpu().numpy()[:n], ref['loss_history'][:n], 1e-3))

if __name__ == '__main__':
    torch.cuda.set_device(0)
    run(30, 100, 1000, chunk=None)
    run(30, 100, 1000, chunk=16, warm=8)
    run(128, 256, 4000, chunk=None)
    run(128, 256, 4000, chunk=64, warm=0)
