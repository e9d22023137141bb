"""Shuffle tests of a fitted model (reference poor_man_gplvm/test.py:1-79).

  * circular_shuffle_data  test.py:10-24  (host generator, as the reference)
  * shuffle_and_decode     test.py:27-45  (device-resident: see below)
  * test_one_model         test.py:48-68
  * compute_entropy        test.py:70-79

shuffle_and_decode draws the shifts exactly as circular_shuffle_data does (numpy's
global RandomState, one np.random.randint(0, n_time) per neuron per shuffle, in the
same order), so a seeded run shuffles the same way as the reference.  The spike
train is uploaded once; each shuffle is one pmg_roll_columns launch into a resident
work buffer, the spike preparation is re-derived in place (SpikeData.refresh) and the
decode runs on one DeviceEM reused for every shuffle, so no per-shuffle allocation,
transition upload or tuning upload happens.  The returned dict stacks every shuffle's
result per key, as the reference does.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _native as nat
from .core import _is_tsd, nap
from .engine import default_device


def _restrict(spk_tsdf, ep):
    if ep is not None:
        if not _is_tsd(spk_tsdf):
            raise TypeError("ep needs a pynapple TsdFrame input (test.py:16-18)")
        spk_tsdf = spk_tsdf.restrict(ep)
    return spk_tsdf


def _shifts(n_time, n_neuron):
    """One shuffle's per-neuron shifts, drawn as test.py:22-23 draws them."""
    return np.array([np.random.randint(0, n_time) for _ in range(n_neuron)], dtype=np.int64)


def circular_shuffle_data(spk_tsdf, n_shuffle=100, ep=None):
    """test.py:10-24: yields n_shuffle copies of the (n_time, n_neuron) spike matrix,
    each neuron's column rolled independently by np.random.randint(0, n_time)."""
    spk_tsdf = _restrict(spk_tsdf, ep)
    y = np.asarray(spk_tsdf.d if _is_tsd(spk_tsdf) else spk_tsdf)
    n_time, n_neuron = y.shape
    for _ in range(n_shuffle):
        s = _shifts(n_time, n_neuron)
        out = np.empty_like(y)
        for j in range(n_neuron):
            out[:, j] = np.roll(y[:, j], s[j])
        yield out


class ShuffleDecoder:
    """Device session for repeated decodes of circularly shuffled copies of one spike
    train with one model: y resident, rolled per shuffle by pmg_roll_columns into the
    engine's own spike buffer."""

    def __init__(self, model, y, decoder_type='naive_bayes', dt_l=1.):
        if decoder_type not in ('naive_bayes', 'dynamics'):
            raise ValueError(f"decoder_type {decoder_type} not supported")
        y = np.asarray(y)
        if y.ndim != 2:
            raise ValueError(f"spike matrix must be (n_time, n_neuron), got {y.shape}")
        self.model, self.decoder_type, self.dt_l = model, decoder_type, dt_l
        self.T, self.N = y.shape
        dev = default_device()
        self.lib = nat.load()
        self.y_src = torch.as_tensor(np.ascontiguousarray(y, dtype=np.float32), device=dev)
        self.y_work = torch.empty_like(self.y_src)
        self.shift = torch.zeros(self.N, dtype=torch.int64, device=dev)
        self.eng = None
        self.hp = model._decode_hp({})

    def _roll(self, shifts):
        s = np.asarray(shifts, dtype=np.int64)
        if s.shape != (self.N,):
            raise ValueError(f"shifts must have shape ({self.N},)")
        self.shift.copy_(torch.as_tensor(s), non_blocking=False)
        nat.check(self.lib.pmg_roll_columns(nat.ptr(self.y_src), self.T, self.N, nat.ptr(self.shift),
                                            nat.ptr(self.y_work), nat.stream_handle()), "pmg_roll_columns")

    # naive-Bayes shuffles decoded per launch: the stacked copies' device bytes stay
    # within this budget (delta, block references, log posterior, ll: ~13 bytes per (t, l))
    NB_BATCH_BYTES = 8 << 30
    NB_BATCH_MAX = 32

    def nb_batch_size(self, n_shuffle):
        per = 13 * self.T * self.model.n_latent_bin + 12 * self.T * self.N
        return int(max(1, min(n_shuffle, self.NB_BATCH_MAX, self.NB_BATCH_BYTES // max(per, 1))))

    def decode_naive_bayes_batch(self, shifts_l):
        """Naive-Bayes decodes of len(shifts_l) shuffles in ONE pass: the rolled copies
        are stacked in time (R T, N), so the spike preparation, the int8-MFMA emission
        and the normaliser each run once for all of them.  Every output row depends on
        its own time bin only, so each returned dict equals decode(shifts) bit for bit."""
        m = self.model
        R = len(shifts_l)
        if R == 1:
            return [self.decode(shifts_l[0])]
        T, N = self.T, self.N
        if getattr(self, '_stack_R', 0) != R:
            self._stack = torch.empty((R * T, N), dtype=torch.float32, device=self.y_src.device)
            self._stack_R = R
            self._stack_eng = None
        for r, s in enumerate(shifts_l):
            s = np.asarray(s, dtype=np.int64)
            if s.shape != (N,):
                raise ValueError(f"shifts must have shape ({N},)")
            self.shift.copy_(torch.as_tensor(s), non_blocking=False)
            nat.check(self.lib.pmg_roll_columns(nat.ptr(self.y_src), T, N, nat.ptr(self.shift),
                                                nat.ptr(self._stack[r * T:(r + 1) * T]), nat.stream_handle()),
                      "pmg_roll_columns")
        if self._stack_eng is None:
            self._stack_eng = m._nb_engine(self._stack, m.tuning, self.hp, m.ma_neuron_default,
                                           m.ma_latent_default)
        else:
            self._stack_eng.sp.refresh()
        return m._nb_on(self._stack_eng, self.dt_l, n_split=R)

    def decode(self, shifts):
        """Decode the copy of y with column j rolled by shifts[j] (np.roll semantics)."""
        m = self.model
        self._roll(shifts)
        if self.decoder_type == 'naive_bayes':
            if self.eng is None:
                self.eng = m._nb_engine(self.y_work, m.tuning, self.hp, m.ma_neuron_default, m.ma_latent_default)
            else:
                self.eng.sp.refresh()
            return m._nb_on(self.eng, self.dt_l)
        hp, logK, logA = m._dynamics_decode_args(self.hp)
        if self.eng is None:
            self.eng = m._decode_engine(self.y_work, m.tuning, hp, m.ma_neuron_default, m.ma_latent_default,
                                        logK, logA)
        else:
            self.eng.sp.refresh()
        r = m._decode_on(self.eng, hp, m.ma_latent_default, 1., True, logK, logA)
        return m._decode_result(r)


def shuffle_and_decode(model, spk_tsdf, n_time_per_chunk=10000, dt_l=1, n_shuffle=100, ep=None,
                       decoder_type='naive_bayes'):
    """test.py:27-45: decode n_shuffle circular shuffles of spk_tsdf with
    decode_latent_naive_bayes ('naive_bayes') or decode_latent ('dynamics'); returns
    {key: np.array over shuffles}.  n_time_per_chunk is accepted and unused (it bounds
    the reference's XLA memory only)."""
    if decoder_type not in ('naive_bayes', 'dynamics'):
        raise ValueError(f"decoder_type {decoder_type} not supported")
    spk_tsdf = _restrict(spk_tsdf, ep)
    y = np.asarray(spk_tsdf.d if _is_tsd(spk_tsdf) else spk_tsdf)
    if n_shuffle < 1:
        raise ValueError("n_shuffle must be >= 1")
    from .model_selection_helper import shard_map
    dec = ShuffleDecoder(model, y, decoder_type, dt_l)
    # every shuffle's shifts drawn first, in the reference's order (the same np.random
    # calls on every rank); the shuffles are then sharded over the torch.distributed ranks
    # when a process group is up, and gathered back in order
    shifts = [_shifts(*y.shape) for _ in range(n_shuffle)]

    def run(idx):
        if decoder_type != 'naive_bayes':
            return [dec.decode(shifts[i]) for i in idx]
        Rg = dec.nb_batch_size(len(idx))      # batched: Rg shuffles decoded per pass
        out = []
        for j in range(0, len(idx), Rg):
            out.extend(dec.decode_naive_bayes_batch([shifts[i] for i in idx[j:j + Rg]]))
        return out
    res_l = shard_map(n_shuffle, run)
    return {k: np.array([d[k] for d in res_l]) for k in res_l[0].keys()}


def test_one_model(y_true, model_fit, n_shuffle=100, decoder_type='naive_bayes', sig_key=None):
    """test.py:48-68: per-time-bin significance of the true decode against the 97.5 %
    quantile of the shuffles.  y_true: pynapple TsdFrame (or an array, times = bin index)."""
    if _is_tsd(y_true):
        t, y = y_true.t, y_true.d
    else:
        y = np.asarray(y_true)
        t = np.arange(y.shape[0], dtype=np.float64)
    if sig_key is None:
        if decoder_type == 'naive_bayes':
            sig_key = 'log_marginal_l'
        elif decoder_type == 'dynamics':
            sig_key = 'log_one_step_predictive_marginals_all'
    if decoder_type == 'naive_bayes':
        res_true = model_fit.decode_latent_naive_bayes(y)
    elif decoder_type == 'dynamics':
        res_true = model_fit.decode_latent(y)
    else:
        raise ValueError(f"decoder_type {decoder_type} not supported")
    res_shuffle = shuffle_and_decode(model_fit, y, n_time_per_chunk=10000, dt_l=1, n_shuffle=n_shuffle, ep=None,
                                     decoder_type=decoder_type)
    log_marg_thresh = np.quantile(res_shuffle[sig_key], 0.975, axis=0)
    is_sig = res_true[sig_key] > log_marg_thresh
    is_sig_tsd = nap.Tsd(d=is_sig, t=t) if nap is not None else {'t': t, 'd': is_sig}
    return {'decode_res_true': res_true, 'decode_res_shuffle': res_shuffle,
            'log_marg_thresh': log_marg_thresh, 'is_sig_tsd': is_sig_tsd}


test_one_model.__test__ = False    # a library function, not a pytest test


def compute_entropy(logp_l, axis=(-1, -2)):
    """test.py:70-79: -sum(p log p) over axis.  States with p = 0 (log p = -inf, which
    this package's log posteriors hold where the reference keeps a very negative finite
    log) contribute 0, the limit of p log p, instead of 0 * -inf = nan."""
    logp_l = np.asarray(logp_l)
    p = np.exp(logp_l)
    with np.errstate(invalid='ignore'):
        plogp = np.where(p > 0, p * logp_l, 0.0)
    return -np.sum(plogp, axis=axis)
