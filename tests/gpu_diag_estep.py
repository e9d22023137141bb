"""Diagnostic (not collected): E-step error sources at the em_c1_fixed iteration-3
tuning: emission error, chunking (warm-up/verify tolerance) and the scan itself."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import gplvm_oracle as O  # noqa: E402


def main():
    from poor_man_gplvm_amd.core import PoissonGPLVMJump1D
    from poor_man_gplvm_amd.engine import ScanConfig
    f = np.load(os.path.join(HERE, 'golden', 'em_c1_fixed.npz'))
    y = f['y'].astype(np.float64)
    ref = O.fit_em(y, f['W0'].astype(np.float64), f['basis'].astype(np.float64), f['lp0'].astype(np.float64),
                   n_iter=3, m_step_maxiter=40, m_step_tol=0.0)
    tun = ref['tuning']
    L = tun.shape[0]
    dref = O.decode_latent(y, tun)
    pre = dref['posterior_latent_marg']
    big = pre > 1e-3
    for chunk, tol, warm in [(None, 1e-6, 64), (400, 1e-6, 64), (32, 1e-9, 64), (32, 1e-6, 256)]:
        m = PoissonGPLVMJump1D(y.shape[1], n_latent_bin=L)
        m.scan_config = ScanConfig(chunk=chunk, warmup=warm, tol=tol)
        dec = m.decode_latent(y.astype(np.float32), tuning=tun)
        pe = dec['posterior_latent_marg']
        r = np.abs(pe - pre) / pre
        tbad = np.argmax(np.max(np.where(big, r, 0), 1))
        lle = np.abs(dec['log_likelihood_all'] - dref['log_likelihood_all'])
        print(f"chunk={chunk} tol={tol} warm={warm}: post rel max {r[big].max():.2e} (t={tbad}) "
              f"med {np.median(r[big]):.2e} | ll abs max {lle.max():.2e} | "
              f"logZ rel {abs(dec['log_marginal_final'] - dref['log_marginal_final']) / abs(dref['log_marginal_final']):.2e}")
    # force the f64 VALU emission (no int8 quantization of log-rates)
    import poor_man_gplvm_amd.engine as E
    orig = E.SpikeData.__init__

    def init_f64(self, *a, **k):
        orig(self, *a, **k)
        self.int_path = False
    E.SpikeData.__init__ = init_f64
    m = PoissonGPLVMJump1D(y.shape[1], n_latent_bin=L)
    dec = m.decode_latent(y.astype(np.float32), tuning=tun)
    E.SpikeData.__init__ = orig
    pe = dec['posterior_latent_marg']
    r2 = np.abs(pe - pre) / pre
    print(f"f64 emission: post rel max {r2[big].max():.2e} med {np.median(r2[big]):.2e} "
          f"logZ rel {abs(dec['log_marginal_final'] - dref['log_marginal_final']) / abs(dref['log_marginal_final']):.2e}")
    rr = np.max(np.where(big, r, 0), 1)
    print("per-t max rel (last config), t with rel>1e-5:", np.nonzero(rr > 1e-5)[0][:40])


if __name__ == '__main__':
    main()
