"""Gradient oracle: float64 torch-CPU autograd restatement of the SMGP ELBO.

TEST INFRASTRUCTURE ONLY (same rule as ``oracle/cpu_ref.py``): only ``tests/``
may import it, as the checker of the HIP backward kernels.  It runs on the CPU
in float64; the product path never imports it.

It follows the same reference semantics as ``cpu_ref.py`` (SURVEY Appendix A,
GPflow 2.7 / TFP 0.18 at the call sites of MixtureGPs/models.py:55-79,
likelihoods.py:39-41, utils.py:26-27), written with differentiable torch ops:
expanded square distance (A.2), Cholesky + triangular solve (A.3), whitened
conditional with band_part(q_sqrt) (A.3), whitened KL (A.4), relaxed one-hot
sample with explicit noise (A.5), Gaussian var-exp (A.6), the SMGP /
SMGPModified ELBO (A.7).  Its value is checked against ``cpu_ref.smgp_elbo`` /
``smgp_modified_elbo`` in tests/test_oracle.py, so the gradients are those of
the pinned forward restatement.
"""
import math

import numpy as np
import torch

JITTER = 1e-6
TAU = 1e-2

LAYER_KEYS = ("Z", "variance", "lengthscales", "q_mu", "q_sqrt")


def _t(x, requires_grad=False):
    t = torch.tensor(np.asarray(x, np.float64), dtype=torch.float64)
    return t.requires_grad_(requires_grad)


def rbf(A, B, variance, lengthscales):
    As, Bs = A / lengthscales, B / lengthscales
    d2 = (As ** 2).sum(-1)[:, None] + (Bs ** 2).sum(-1)[None, :] - 2.0 * As @ Bs.T
    return variance * torch.exp(-0.5 * d2)


def layer_conditional(X, L):
    """Whitened SVGP marginals (models.py:129-144): fmean, fvar [N, K] and A [M, N]."""
    Z = L["Z"]
    M = Z.shape[0]
    Kuu = rbf(Z, Z, L["variance"], L["lengthscales"]) + JITTER * torch.eye(M, dtype=Z.dtype)
    Lm = torch.linalg.cholesky(Kuu)
    Kuf = rbf(Z, X, L["variance"], L["lengthscales"])
    A = torch.linalg.solve_triangular(Lm, Kuf, upper=False)
    fmean = A.T @ L["q_mu"]
    Lk = torch.tril(L["q_sqrt"])
    LTA = Lk.transpose(1, 2) @ A                                  # [K, M, N]
    fvar = L["variance"] - (A ** 2).sum(0)[:, None] + (LTA ** 2).sum(1).T
    return fmean, fvar, A


def gauss_kl_white(q_mu, q_sqrt):
    L = torch.tril(q_sqrt)
    d = torch.diagonal(L, dim1=1, dim2=2)
    return 0.5 * ((q_mu ** 2).sum() - q_mu.numel() - torch.log(d ** 2).sum() + (L ** 2).sum())


def _var_exp(mu, var, y, lik_var):
    return -0.5 * math.log(2 * math.pi) - 0.5 * torch.log(lik_var) - 0.5 * ((y - mu) ** 2 + var) / lik_var


_GH_X, _GH_W = np.polynomial.hermite.hermgauss(20)


def multiclass_var_exp(mu, var, Y, eps):
    """GPflow 2.7.0 MultiClass/RobustMax var-exp (cpu_ref.multiclass_var_exp) on
    [N, K] latents -> [N] (differentiable)."""
    N, K = mu.shape
    y = torch.as_tensor(np.asarray(Y).reshape(-1).astype(np.int64))
    oh_on = torch.zeros(N, K, dtype=mu.dtype)
    ok = (y >= 0) & (y < K)
    oh_on[torch.nonzero(ok).reshape(-1), y[ok]] = 1.0
    ss = lambda v: torch.sqrt(torch.clamp(v, min=1e-10))
    mu_sel, var_sel = (oh_on * mu).sum(1), (oh_on * var).sum(1)
    X = mu_sel[:, None] + torch.as_tensor(_GH_X) * ss(2.0 * var_sel)[:, None]
    dist = (X[:, None, :] - mu[:, :, None]) / ss(var)[:, :, None]
    cdfs = 0.5 * (1.0 + torch.erf(dist / math.sqrt(2.0)))
    cdfs = cdfs * (1 - 2e-6) + 1e-6
    cdfs = cdfs * (1.0 - oh_on)[:, :, None] + oh_on[:, :, None]
    p = torch.prod(cdfs, 1) @ torch.as_tensor(_GH_W / np.sqrt(np.pi)).reshape(-1, 1)
    return (p * math.log(1.0 - eps) + (1.0 - p) * math.log(eps / (K - 1.0))).sum(-1)


def _pred_ve(mu_f, var_f, Y, lik_var, multiclass_eps):
    """[1, N, K] Gaussian var-exp or [1, N, 1] MultiClass var-exp (S-invariant)."""
    if multiclass_eps is not None:
        return multiclass_var_exp(mu_f, var_f, Y, multiclass_eps).reshape(1, -1, 1)
    return _var_exp(mu_f[None], var_f[None], Y.reshape(1, -1, 1), lik_var)


def data_term(mu_f, var_f, mu_a, var_a, Y, lik_var, z, u, assign_lik_var=None, multiclass_eps=None):
    """sum_n DT_n (models.py:55-67,73-74; SMGPModified :112-123 with assign_lik_var)
    as a function of the conditionals [N, K] (the K6 boundary)."""
    S = z.shape[0]
    y = Y.reshape(1, -1, 1)
    logits = mu_a[None] + z * torch.sqrt(var_a[None] + 1e-6)
    g = -torch.log(-torch.log(u))
    W = torch.softmax((g + logits) / TAU, dim=-1)
    ve = _pred_ve(mu_f, var_f, Y, lik_var, multiclass_eps)
    data = torch.logsumexp((W * ve).sum(2), 0) - math.log(S)
    if assign_lik_var is not None:
        vea = _var_exp(mu_a[None], var_a[None], y, assign_lik_var)
        data = data + torch.logsumexp((W * vea).sum(2), 0) - math.log(S)
    return data.sum()


def elbo(X, Y, pred, assign, lik_var, z, u, num_data, assign_lik_var=None, keep=None, multiclass_eps=None):
    """SMGP (or SMGPModified when assign_lik_var is given) ELBO, float64 scalar.
    pred/assign: dicts of tensors (LAYER_KEYS); lik_var [K]; z, u [S, N, K].
    keep: optional dict that receives the conditional tensors (retain_grad set)."""
    S = z.shape[0]
    mu_f, var_f, _ = layer_conditional(X, pred)
    mu_a, var_a, _ = layer_conditional(X, assign)
    if keep is not None:
        for name, t in (("mu_f", mu_f), ("var_f", var_f), ("mu_a", mu_a), ("var_a", var_a)):
            t.retain_grad()
            keep[name] = t
    y = Y.reshape(1, -1, 1)
    logits = mu_a[None] + z * torch.sqrt(var_a[None] + 1e-6)
    g = -torch.log(-torch.log(u))
    W = torch.softmax((g + logits) / TAU, dim=-1)
    ve = _pred_ve(mu_f, var_f, Y, lik_var, multiclass_eps)
    data = torch.logsumexp((W * ve).sum(2), 0) - math.log(S)
    if assign_lik_var is not None:
        vea = _var_exp(mu_a[None], var_a[None], y, assign_lik_var)
        data = data + torch.logsumexp((W * vea).sum(2), 0) - math.log(S)
    kl = gauss_kl_white(pred["q_mu"], pred["q_sqrt"]) + gauss_kl_white(assign["q_mu"], assign["q_sqrt"])
    return data.mean() - kl / num_data


def params_from_oracle(p, requires_grad=True):
    """cpu_ref.SMGPParams -> (pred, assign, lik_var) dicts of float64 leaf tensors
    (values rounded through float32, as the device model holds them)."""
    def layer(L):
        out = {}
        for k in LAYER_KEYS:
            v = np.asarray(L[k], np.float64).astype(np.float32).astype(np.float64)
            if k == "lengthscales":
                v = np.atleast_1d(v)
            out[k] = _t(v, requires_grad)
        return out
    lik = _t(np.asarray(p.lik_variance, np.float64).reshape(-1).astype(np.float32), requires_grad)
    return layer(p.pred), layer(p.assign), lik
