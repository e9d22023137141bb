"""Host-side kernels, basis and transition description (built once per fit).

Restates, in numpy, the parts of the reference that run once per model / fit:
  * generate_basis              core.py:41-73
  * create_transition_prob_1d   gp_kernel.py:42-89 (rbf_kernel :14-20,
                                 uniform_kernel :36-40, discrete_transition_kernel :30-34)
and derives the device form of the continuous transition kernel:
  * BandedTransition: the row-normalised RBF K0[i,j] = g[|i-j|] / Z_i is Toeplitz up
    to the row scale and negligible beyond |i-j| = band (g[band+1] < 1e-30 * g[0]), so
    the linear-space scans (fb_kernels.h) receive (g[0..band], 1/Z), band <= 32;
  * DenseTransition: any other continuous kernel (custom_transition_kernel, wider RBF
    kernels, and the latent-only model, whose far moves carry weights below the fp32 /
    f64 range) as the full (L, L) log kernel for the log-domain scans (dense_scan.hip).
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
    if n_latent_bin > 1024:
        raise NotImplementedError("the banded scans hold n_latent_bin <= 1024 (larger: the dense scans)")
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


@dataclass
class DenseTransition:
    """Full log-domain device description: logK0 (L, L) [i_prev, j_next] (row-normalised,
    -inf allowed), uniform jump kernel, dynamics A (2, 2)."""
    L: int
    logK0: np.ndarray    # (L, L) float64
    A: np.ndarray        # (2, 2) float64
    movement_variance: float = float('nan')
    band: int = -1       # (no band: the dense scans hold the whole kernel)

    @property
    def logA(self):
        return _get_log(self.A)


def dense_transition(n_latent_bin, movement_variance=1.0, p_move_to_jump=0.01, p_jump_to_move=0.01,
                     custom_kernel=None) -> DenseTransition:
    """create_transition_prob_1d (gp_kernel.py:42-89) for the dense log-domain scans."""
    _, logK, A, _ = create_transition_prob_1d(n_latent_bin, movement_variance, p_move_to_jump, p_jump_to_move,
                                              custom_kernel)
    mv = float(movement_variance) if custom_kernel is None else float('nan')
    return DenseTransition(L=int(n_latent_bin), logK0=logK[0], A=A, movement_variance=mv)


def make_transition(n_latent_bin, movement_variance=1.0, p_move_to_jump=0.01, p_jump_to_move=0.01,
                    custom_kernel=None):
    """The scan transition for these hyper-parameters: banded (fast linear-space
    scans) when the continuous kernel has the <= 32-bin Toeplitz form, else dense."""
    if custom_kernel is None:
        try:
            return banded_transition(n_latent_bin, movement_variance, p_move_to_jump, p_jump_to_move)
        except NotImplementedError:
            pass
    return dense_transition(n_latent_bin, movement_variance, p_move_to_jump, p_jump_to_move, custom_kernel)


def transition_from_log_kernels(log_latent_transition_kernel_l, log_dynamics_transition_kernel,
                                rtol=1e-6, force_dense=False):
    """Device form of arbitrary kernels in the reference's layout (the arguments of
    _decode_latent, core.py:777-786): logK (2, L, L) [d_next, i_prev, j_next], logA (2, 2).

    The banded scans hold the continuous kernel as a row-scaled Toeplitz band
    K0[i, j] = g[|i-j|] * invz[i] and the jump kernel as uniform 1/L.  This recovers
    (g, invz, band) from K0 = exp(logK[0]) and checks that it reproduces every entry to
    rtol of its row maximum, with the entries beyond the band below 1e-30 of it; any
    other continuous kernel is returned whole for the dense log-domain scans.  A jump
    kernel that is not uniform raises NotImplementedError (the reference never builds
    one, gp_kernel.py:36-40)."""
    lk = np.asarray(log_latent_transition_kernel_l, np.float64)
    la = np.asarray(log_dynamics_transition_kernel, np.float64)
    if lk.ndim != 3 or lk.shape[0] != 2 or lk.shape[1] != lk.shape[2] or la.shape != (2, 2):
        raise ValueError(f"expected logK (2, L, L) and logA (2, 2), got {lk.shape} and {la.shape}")
    L = lk.shape[1]
    K = np.exp(lk)
    if not np.allclose(K[1], 1.0 / L, rtol=rtol, atol=0.0):
        raise NotImplementedError("jump kernel (logK[1]) is not uniform 1/L: not supported by the scan kernels")
    K0 = K[0]
    rowmax = K0.max(axis=1)
    if not np.all(rowmax > 0):
        raise ValueError("continuous kernel has an all-zero row")
    dense = DenseTransition(L=L, logK0=lk[0].copy(), A=np.exp(la))
    if force_dense or L > 1024:     # the banded scans hold L <= 1024
        return dense
    dia = np.diagonal(K0)
    if not np.all(dia >= rowmax * (1 - rtol)):
        return dense
    c = L // 2
    gfull = K0[c, c:] / K0[c, c]                      # g[k] for k = 0 .. L-1-c (centre row)
    gl = K0[c, :c + 1][::-1] / K0[c, c]
    gfull = gfull if gfull.size >= gl.size else gl
    nz = np.flatnonzero(gfull > BAND_REL_CUTOFF)
    band = int(nz.max()) if nz.size else 0
    if band > MAX_BAND:
        return dense
    g = gfull[:band + 1]
    invz = dia.copy()
    i = np.arange(L)
    dist = np.abs(i[:, None] - i[None, :])
    recon = np.where(dist <= band, g[np.minimum(dist, band)] * invz[:, None], 0.0)
    if np.max(np.abs(recon - K0) / rowmax[:, None]) > rtol:
        return dense
    A = np.exp(la)
    mv = float('nan')
    if band >= 1 and 0 < g[1] < 1:
        mv = float(1.0 / math.sqrt(-math.log(g[1])))  # g[1] = exp(-1/mv^2) for the RBF kernel
    return BandedTransition(L=L, band=band, g=g.astype(np.float32), invz=invz.astype(np.float32),
                            A=A, movement_variance=mv)
