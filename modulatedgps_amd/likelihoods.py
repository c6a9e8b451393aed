"""GaussianModified likelihood (MixtureGPs/likelihoods.py:12-41) and GPflow's
MultiClass / RobustMax (the pred likelihood of the multiclass demos,
demos/demo_tf2_modified_multiclass.py:43-45) on the device.

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


# 20-point Gauss-Hermite rule of gpflow.quadrature.hermgauss (numpy hermgauss).
_GH_X, _GH_W = np.polynomial.hermite.hermgauss(20)


class RobustMax:
    """gpflow.likelihoods.RobustMax (GPflow 2.7.0, pinned at environment.yml:95):
    the robust-max inverse link with epsilon (default 1e-3, a non-trainable
    parameter in GPflow) and the 1e-6 CDF squash of prob_is_largest."""

    def __init__(self, num_classes: int, epsilon: float = 1e-3, device=None):
        if num_classes < 2:
            raise ValueError("RobustMax needs num_classes >= 2")
        if not (0.0 < epsilon < 1.0):
            raise ValueError("epsilon must lie in (0, 1)")
        self.num_classes = int(num_classes)
        self.epsilon = float(epsilon)
        self._squash = 1e-6
        self.device = torch.device(device or default_device())

    @property
    def eps_k1(self):
        return self.epsilon / (self.num_classes - 1.0)

    def __call__(self, F):
        """one_hot(argmax F, K, 1 - eps, eps / (K - 1))."""
        i = torch.argmax(F, -1)
        out = torch.full(F.shape, self.eps_k1, dtype=F.dtype, device=F.device)
        return out.scatter_(-1, i.unsqueeze(-1), 1.0 - self.epsilon)

    @staticmethod
    def safe_sqrt(v):
        return torch.sqrt(torch.clamp(v, min=1e-10))

    def prob_is_largest(self, Y, mu, var, gh_x=_GH_X, gh_w=_GH_W):
        """P(latent Y is the largest) under independent N(mu_k, var_k): [N, 1]."""
        Y = torch.as_tensor(Y, device=mu.device).reshape(-1).to(torch.int64)
        K = self.num_classes
        valid = (Y >= 0) & (Y < K)
        oh_on = torch.zeros(mu.shape[0], K, dtype=mu.dtype, device=mu.device)
        oh_on[valid] = torch.nn.functional.one_hot(Y[valid], K).to(mu.dtype)
        mu_sel = (oh_on * mu).sum(1)
        var_sel = (oh_on * var).sum(1)
        gx = torch.as_tensor(gh_x, dtype=mu.dtype, device=mu.device)
        gw = torch.as_tensor(gh_w / np.sqrt(np.pi), dtype=mu.dtype, device=mu.device)
        X = mu_sel[:, None] + gx * self.safe_sqrt(2.0 * var_sel)[:, None]
        dist = (X[:, None, :] - mu[:, :, None]) / self.safe_sqrt(var)[:, :, None]
        cdfs = 0.5 * (1.0 + torch.erf(dist / math.sqrt(2.0)))
        cdfs = cdfs * (1 - 2 * self._squash) + self._squash
        cdfs = cdfs * (1.0 - oh_on)[:, :, None] + oh_on[:, :, None]
        return torch.prod(cdfs, 1) @ gw.reshape(-1, 1)


class MultiClass:
    """gpflow.likelihoods.MultiClass(num_classes, invlink=RobustMax) (GPflow 2.7.0).

    In the ELBO the var-exp is fused into K6 (mgp_elbo_terms_multiclass) and the
    predictive moments into mgp_multiclass_predict; these methods keep GPflow's
    names and semantics on arbitrary device tensors ([N, K] latents, Y [N, 1])."""

    def __init__(self, num_classes: int, invlink: RobustMax = None, device=None):
        self.num_classes = int(num_classes)
        self.num_gauss_hermite_points = 20
        self.invlink = invlink if invlink is not None else RobustMax(self.num_classes, device=device)
        if not isinstance(self.invlink, RobustMax):
            raise NotImplementedError("MultiClass supports the RobustMax inverse link only (as GPflow)")
        if self.invlink.num_classes != self.num_classes:
            raise ValueError("invlink.num_classes must equal num_classes")
        self.device = self.invlink.device

    def _log_prob(self, X, F, Y):
        hits = torch.argmax(F, 1, keepdim=True) == torch.as_tensor(Y, device=F.device).to(torch.int64)
        p = torch.where(hits, 1.0 - self.invlink.epsilon, self.invlink.eps_k1).to(F.dtype)
        return torch.log(p).sum(-1)

    def _variational_expectations(self, X, Fmu, Fvar, Y):
        p = self.invlink.prob_is_largest(Y, Fmu, Fvar)
        ve = p * math.log(1.0 - self.invlink.epsilon) + (1.0 - p) * math.log(self.invlink.eps_k1)
        return ve.sum(-1)

    def _predict_non_logged_density(self, X, Fmu, Fvar, Y):
        p = self.invlink.prob_is_largest(Y, Fmu, Fvar)
        return p * (1.0 - self.invlink.epsilon) + (1.0 - p) * self.invlink.eps_k1

    def _predict_mean_and_var(self, X, Fmu, Fvar):
        N = Fmu.shape[0]
        ps = torch.cat([self._predict_non_logged_density(
            X, Fmu, Fvar, torch.full((N, 1), i, dtype=torch.int64, device=Fmu.device))
            for i in range(self.num_classes)], 1)
        return ps, ps - ps ** 2

    def _predict_log_density(self, X, Fmu, Fvar, Y):
        return torch.log(self._predict_non_logged_density(X, Fmu, Fvar, Y)).sum(-1)

    def _conditional_mean(self, X, F):
        return self.invlink(F)

    def _conditional_variance(self, X, F):
        p = self._conditional_mean(X, F)
        return p - p ** 2

    def __repr__(self):
        return f"MultiClass(num_classes={self.num_classes}, epsilon={self.invlink.epsilon})"
