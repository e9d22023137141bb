"""Host logic of poor_man_gplvm_amd.test (reference test.py:10-79): the shuffles are the
reference's own draws (same global-RandomState sequence, same np.roll direction), and
compute_entropy matches the oracle.  No GPU needed."""
import numpy as np
import pytest

from oracle import gplvm_oracle as O
from poor_man_gplvm_amd import test as PT


def test_circular_shuffle_matches_reference_draws():
    y = np.arange(37 * 5, dtype=np.float32).reshape(37, 5)
    np.random.seed(12)
    ours = list(PT.circular_shuffle_data(y, n_shuffle=4))
    np.random.seed(12)
    for got in ours:
        want, _ = O.circular_shuffle_once(y)
        np.testing.assert_array_equal(got, want)
    # every column is a rotation of the original column
    for got in ours:
        for j in range(5):
            k = int(np.flatnonzero(got[:, j] == y[0, j])[0])
            np.testing.assert_array_equal(got[:, j], np.roll(y[:, j], k))


def test_shift_sequence_matches_reference():
    np.random.seed(3)
    s = [PT._shifts(100, 7) for _ in range(3)]
    np.random.seed(3)
    for got in s:
        _, want = O.circular_shuffle_once(np.zeros((100, 7)))
        np.testing.assert_array_equal(got, want)
        assert got.min() >= 0 and got.max() < 100


def test_compute_entropy():
    rng = np.random.default_rng(0)
    p = rng.dirichlet(np.ones(12), size=(9, 2)).reshape(9, 2, 12)
    p /= p.sum(axis=(-1, -2), keepdims=True)
    lp = np.log(p)
    np.testing.assert_allclose(PT.compute_entropy(lp), O.compute_entropy(lp), rtol=1e-12)
    np.testing.assert_allclose(PT.compute_entropy(lp), -(p * lp).sum(axis=(-1, -2)), rtol=1e-12)
    lp2 = lp.copy()
    lp2[:, :, 0] = -np.inf          # zero-probability states contribute 0
    e = PT.compute_entropy(lp2)
    assert np.all(np.isfinite(e))
    np.testing.assert_allclose(e, -(p[:, :, 1:] * lp[:, :, 1:]).sum(axis=(-1, -2)), rtol=1e-12)
    assert PT.compute_entropy(lp[0, 0], axis=-1).shape == ()


def test_shuffle_and_decode_rejects_bad_decoder():
    with pytest.raises(ValueError):
        PT.shuffle_and_decode(None, np.zeros((10, 3)), decoder_type='viterbi')
    with pytest.raises(TypeError):
        PT.shuffle_and_decode(None, np.zeros((10, 3)), ep=(0, 1))
