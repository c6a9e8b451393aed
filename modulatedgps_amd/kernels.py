"""SquaredExponential kernel (drop-in for gpflow.kernels.SquaredExponential as used by
the reference demos, e.g. demos/demo_tf2.py:37-38) backed by the gfx950 RBF kernels.

Hyper-parameters are stored as constrained float32 device tensors (variance [1],
lengthscales [1] or [D]); the kernels read them through device pointers so no
call synchronises with the host.
"""
import numpy as np
import torch

from . import ops
from .config import default_device, default_jitter


def _param(v, device):
    t = torch.as_tensor(np.asarray(v, dtype=np.float32).reshape(-1), device=device)
    return t.clone()


class SquaredExponential:
    """k(x, x') = variance * exp(-0.5 * ||(x - x') / lengthscales||^2)."""

    def __init__(self, variance=1.0, lengthscales=1.0, device=None):
        dev = device or default_device()
        self.device = torch.device(dev)
        if np.any(np.asarray(variance) <= 0) or np.any(np.asarray(lengthscales) <= 0):
            raise ValueError("variance and lengthscales must be positive")
        self.variance = _param(variance, self.device)
        self.lengthscales = _param(lengthscales, self.device)

    # GPflow-style API ---------------------------------------------------------------
    def K(self, A, B=None):
        """K(A, B) [M_A, N_B] (models.py:139 calls K(Z, Xnew))."""
        A = self._x(A)
        if B is None:
            return ops.rbf_kuu(A, self.variance, self.lengthscales, 0.0)
        return ops.rbf_kuf(self._x(B), A, self.variance, self.lengthscales)

    def Kuu(self, Z, jitter=None):
        """covariances.Kuu(Z, kernel, jitter) (models.py:135)."""
        return ops.rbf_kuu(self._x(Z), self.variance, self.lengthscales,
                           default_jitter() if jitter is None else jitter)

    def K_diag(self, X):
        """Stationary.K_diag: variance broadcast to X.shape[:-1] (models.py:133)."""
        X = torch.as_tensor(X)
        return self.variance.expand(X.shape[:-1])

    def __call__(self, X, X2=None, full_cov=True):
        if not full_cov:
            return self.K_diag(X)
        return self.K(X, X2)

    def _x(self, X):
        """Inputs as float32 device rows with unit innermost stride (numpy views such
        as linspace(...)[:, None] carry a 0 stride on the size-1 axis)."""
        X = torch.as_tensor(X)
        if X.dim() == 1:
            X = X[:, None]
        if X.dtype != torch.float32 or X.device != self.device or X.stride(-1) != 1:
            X = torch.empty(X.shape, dtype=torch.float32, device=self.device).copy_(X)
        return X

    def parameters(self):
        return {"variance": self.variance, "lengthscales": self.lengthscales}

    def __repr__(self):
        return (f"SquaredExponential(variance={self.variance.tolist()}, "
                f"lengthscales={self.lengthscales.tolist()})")
