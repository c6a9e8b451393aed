"""GaussianModified likelihood (MixtureGPs/likelihoods.py:12-41) on the device.

The per-expert noise variance is a [1, K] parameter (likelihoods.py:16-19).  The
ELBO and predict_y hot paths never call these methods: the var-exp is fused
into mgp_elbo_terms and the predictive epilogue into mgp_predict_epilogue.  The
methods are kept (same names, same argument meaning) for API parity and act on
arbitrary device tensors with broadcasting.
"""
import math

import numpy as np
import torch

from .config import default_device


class GaussianModified:
    def __init__(self, variance=1.0, D: int = None, device=None):
        dev = torch.device(device or default_device())
        v = np.asarray(variance, dtype=np.float64)
        if D is not None:
            v = v * np.ones((1, D))                                 # likelihoods.py:16-17
        v = np.atleast_2d(v)
        if np.any(v <= 0):
            raise ValueError("variance must be positive")
        self.variance = torch.as_tensor(v, dtype=torch.float32, device=dev).contiguous()
        self.device = dev

    @property
    def num_experts(self):
        return self.variance.shape[-1]

    def _scalar_log_prob(self, X, F, Y):
        """logdensities.gaussian(Y, F, var) (likelihoods.py:21-22)."""
        v = self.variance
        return -0.5 * (math.log(2 * math.pi) + torch.log(v) + (F - Y) ** 2 / v)

    def _conditional_mean(self, X, F):
        return F.clone()

    def _conditional_variance(self, X, F):
        return self.variance.expand_as(F)

    def _predict_mean_and_var(self, X, Fmu, Fvar):
        """likelihoods.py:31-32."""
        return Fmu.clone(), Fvar + self.variance

    def _predict_log_density(self, X, Fmu, Fvar, Y):
        v = Fvar + self.variance
        return torch.sum(-0.5 * (math.log(2 * math.pi) + torch.log(v) + (Fmu - Y) ** 2 / v), -1)

    def _variational_expectations(self, X, Fmu, Fvar, Y):
        """likelihoods.py:39-41."""
        v = self.variance
        return -0.5 * math.log(2 * math.pi) - 0.5 * torch.log(v) - 0.5 * ((Y - Fmu) ** 2 + Fvar) / v

    def __repr__(self):
        return f"GaussianModified(variance={self.variance.tolist()})"
