"""Host-side kernels, basis and transition description (built once per fit).

Restates, in numpy, the parts of the reference that run once per model / fit:
  * generate_basis              core.py:41-73
  * create_transition_prob_1d   gp_kernel.py:42-89 (rbf_kernel :14-20,
                                 uniform_kernel :36-40, discrete_transition_kernel :30-34)
and derives the compact device form of the continuous transition kernel: the
row-normalised RBF K0[i,j] = g[|i-j|] / Z_i is Toeplitz up to the row scale and
exactly negligible beyond |i-j| = band (g[band+1] < 1e-30 * g[0]), so the device
kernels receive (g[0..band], 1/Z) instead of an L x L matrix.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

BAND_REL_CUTOFF = 1e-30
MAX_BAND = 32


def rbf_kernel_matrix(n, ls, var=1.0, dtype=np.float64):
    """gp_kernel.py:14-20 over all pairs: (val, log_val)."""
    x = np.arange(n, dtype=dtype)
    d2 = (x[:, None] - x[None, :]) ** 2
    val = np.exp(-d2 / dtype(ls) ** 2) * dtype(var)
    logval = -d2 / dtype(ls) ** 2 + np.log(dtype(var))
    return val, logval


def generate_basis(lengthscale, n_latent_bin, explained_variance_threshold_basis=0.999,
                   include_bias=True, basis_type='rbf', custom_kernel=None):
    """core.py:41-73: SVD of the (float32) RBF tuning kernel; keep the columns
    up to the explained-variance threshold scaled by S^(1/4); prepend ones."""
    if custom_kernel is not None:
        basis_type = 'custom_kernel'
    if basis_type == 'rbf':
        kmat, _ = rbf_kernel_matrix(n_latent_bin, lengthscale, 1.0, dtype=np.float32)
    elif basis_type == 'custom_kernel':
        kmat = np.asarray(custom_kernel, dtype=np.float32)
    else:
        raise ValueError(f"basis_type {basis_type!r} not supported (the reference removed bspline, core.py:57-59)")
    u, s, _ = np.linalg.svd(kmat)
    n_basis = int((np.cumsum(s / s.sum()) < explained_variance_threshold_basis).sum()) + 1
    basis = u[:, :n_basis] * np.sqrt(np.sqrt(s))[:n_basis][None, :]
    if include_bias:
        basis = np.concatenate([np.ones((n_latent_bin, 1), dtype=basis.dtype), basis], axis=1)
    return basis.astype(np.float32)


def _get_log(v):
    """gp_kernel.py:8-12."""
    with np.errstate(divide='ignore'):
        lv = np.log(v)
    return np.where(lv == np.inf, -10000.0, lv)


def create_transition_prob_1d(n_latent_bin, movement_variance=1.0, p_move_to_jump=0.01,
                              p_jump_to_move=0.01, custom_kernel=None):
    """gp_kernel.py:42-89 -> (K (2,L,L), logK (2,L,L), A (2,2), logA (2,2)) in
    float64; logK[d_next, i_prev, j_next] with rows normalised over j."""
    L = int(n_latent_bin)
    if custom_kernel is None:
        k0, lk0 = rbf_kernel_matrix(L, movement_variance)
    else:
        k0 = np.asarray(custom_kernel, np.float64)
        lk0 = _get_log(k0)
    k1 = np.full((L, L), 1.0 / L)
    lk1 = np.full((L, L), math.log(1.0 / L))
    K, logK = [], []
    for k, lk in ((k0, lk0), (k1, lk1)):
        z = k.sum(1, keepdims=True)
        K.append(k / z)
        logK.append(lk - np.log(z))
    A = np.array([[1 - p_move_to_jump, p_move_to_jump], [p_jump_to_move, 1 - p_jump_to_move]], np.float64)
    return np.array(K), np.array(logK), A, _get_log(A)


@dataclass
class BandedTransition:
    """Device description of create_transition_prob_1d's output."""
    L: int
    band: int
    g: np.ndarray        # (band+1,) float32
    invz: np.ndarray     # (L,) float32
    A: np.ndarray        # (2,2) float64
    movement_variance: float

    @property
    def logA(self):
        return _get_log(self.A)


def banded_transition(n_latent_bin, movement_variance=1.0, p_move_to_jump=0.01,
                      p_jump_to_move=0.01, custom_kernel=None) -> BandedTransition:
    """Compact (Toeplitz band + row normaliser) form of the continuous kernel."""
    if custom_kernel is not None:
        raise NotImplementedError(
            "custom_transition_kernel (a dense L x L continuous kernel, gp_kernel.py:61-66) is not "
            "supported by the banded device kernels yet")
    L = int(n_latent_bin)
    mv = float(movement_variance)
    if not mv > 0:
        raise ValueError("movement_variance must be > 0")
    band = min(L - 1, int(math.ceil(math.sqrt(-math.log(BAND_REL_CUTOFF)) * mv)))
    if band > MAX_BAND:
        raise NotImplementedError(
            f"movement_variance={mv} needs a continuous-kernel band of {band} > {MAX_BAND} latent bins; "
            "wide / dense kernels are not supported by the device kernels yet")
    k = np.arange(band + 1, dtype=np.float64)
    g = np.exp(-(k ** 2) / mv ** 2)
    x = np.arange(L, dtype=np.float64)
    z = np.exp(-((x[:, None] - x[None, :]) ** 2) / mv ** 2).sum(1)   # full-row normaliser (gp_kernel.py:76)
    A = np.array([[1 - p_move_to_jump, p_move_to_jump], [p_jump_to_move, 1 - p_jump_to_move]], np.float64)
    return BandedTransition(L=L, band=band, g=g.astype(np.float32), invz=(1.0 / z).astype(np.float32),
                            A=A, movement_variance=mv)
