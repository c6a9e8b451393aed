"""Toy data generators of the demos: drop-in for the reference's
utils/dataset_utils.py:84-166 (same names, signatures and random-stream
consumption, so the same numpy Generator gives bit-identical arrays; checked
against fixtures made by the reference's own functions,
tests/golden/toy_datasets.npz).  The John-Doe loaders (:8-81) read the
reference's CSV files and are outside this build."""
import numpy as np


def _flip_labels(rng, labels, fraction):
    """Turn a random `fraction` of the binary labels into outliers (in place)."""
    n = labels.shape[0]
    picked = rng.choice(n, size=int(n * fraction), replace=False)
    labels[picked] = 1 - labels[picked]
    return labels


def load_toy_data_categorical(rng: np.random.Generator):
    """1-D two-class data: label 1 left of the origin, 10 % flipped (dataset_utils.py:84-97)."""
    n, n_test, lo, hi = 500, 100, -6.0, 6.0
    X = rng.uniform(low=lo, high=hi, size=(n, 1))
    Y = _flip_labels(rng, np.where(X < 0.0, 1, 0), 0.1)
    return n, X, Y, np.linspace(lo, hi, n_test).reshape(n_test, 1)


def load_toy_multimodal_data(rng: np.random.Generator):
    """Three 1-D regimes of 500 points each sharing one noise draw (dataset_utils.py:100-114)."""
    n, n_test = 1500, 100
    third = n // 3
    noise = rng.normal(0, 0.1, (third, 1))
    X = rng.uniform(low=-2 * np.pi, high=2 * np.pi, size=(n, 1))
    a, b, c = X[:third], X[third:2 * third], X[2 * third:]
    Y = np.concatenate((np.sin(a) + noise,
                        np.sin(b) - 2 * np.exp(-0.5 * pow(b - 2, 2)) + noise,
                        -2 - (3 / (8 * np.pi)) * c + (3 / 10) * np.sin(2 * c) + noise))
    return n, X, Y, np.linspace(-2 * np.pi, 2 * np.pi, n_test)[:, None]


def load_toy_data_assoc():
    """Data-association toy set on numpy's global RNG (dataset_utils.py:117-125)."""
    n, n_test, outlier_rate = 500, 100, .4
    is_outlier = np.random.binomial(1, outlier_rate, size=(n, 1))
    noise = np.random.randn(n, 1) * .15
    clutter = np.random.uniform(low=-1., high=3., size=(n, 1))
    X = np.random.uniform(low=-3., high=3., size=(n, 1))
    signal = np.cos(.5 * np.pi * X) * np.exp(-.25 * X ** 2) + noise
    Y = (1. - is_outlier) * signal + is_outlier * clutter
    return n, X, Y, np.linspace(-3, 3, n_test)[:, None]


def _radius(X):
    return np.sqrt((X[:, 0] - 0.5) ** 2 + (X[:, 1] - 0.5) ** 2)


def load_toy_2d_data(rng: np.random.Generator):
    """2-D radial surface, the second half lifted by 10 (dataset_utils.py:128-146)."""
    n, n_test = 500, 100
    lo, hi = [-12.0, -12.0], [12.0, 12.0]
    X = rng.uniform(low=lo, high=hi, size=(n, 2))
    r = _radius(X)
    Y = np.concatenate((r[:n // 2], (r + 10.0)[n // 2:])).reshape((n, 1))
    return n, X, Y, np.linspace(lo, hi, n_test)


def load_toy_2d_data_categorical(rng: np.random.Generator):
    """2-D two-class data: label 1 in the negative quadrant, 10 % flipped (dataset_utils.py:149-166)."""
    n, n_test = 500, 100
    lo, hi = [-6.0, -6.0], [6.0, 6.0]
    X = rng.uniform(low=lo, high=hi, size=(n, 2))
    Y = _flip_labels(rng, np.where((X[:, 0] < 0) & (X[:, 1] < 0), 1, 0), 0.1).reshape((n, 1))
    return n, X, Y, np.linspace(lo, hi, n_test)
