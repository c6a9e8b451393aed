"""BroadcastingLikelihood (MixtureGPs/broadcasting_lik.py:5-46).

Lifts a likelihood over the Monte-Carlo sample axis S: inputs [S, N, D], Y [N, D].
For GaussianModified Y is only expanded to [1, N, D] (broadcasting_lik.py:17-18,
23-24); other likelihoods go through the flatten-to-[S*N, D] path (:25-37).
"""
import torch

from .likelihoods import GaussianModified


class BroadcastingLikelihood:
    def __init__(self, likelihood):
        self.likelihood = likelihood
        self.needs_broadcasting = not isinstance(likelihood, GaussianModified)

    def _broadcast(self, f, vars_SND, vars_ND):
        if not self.needs_broadcasting:
            return f(vars_SND, [v.unsqueeze(0) for v in vars_ND])
        S, N, D = vars_SND[0].shape
        vars_tiled = [x.unsqueeze(0).expand(S, *x.shape) for x in vars_ND]
        flattened_SND = [x.reshape(S * N, D) for x in vars_SND]
        flattened_tiled = [x.reshape(S * N, -1) for x in vars_tiled]
        res = f(flattened_SND, flattened_tiled)
        if isinstance(res, (tuple, list)):
            return [x.reshape(S, N, -1) for x in res]
        return res.reshape(S, N, -1)

    def variational_expectations(self, X, Fmu, Fvar, Y):
        f = lambda SND, ND: self.likelihood._variational_expectations([], SND[0], SND[1], ND[0])
        return self._broadcast(f, [Fmu, Fvar], [torch.as_tensor(Y, device=Fmu.device, dtype=Fmu.dtype)])

    def predict_mean_and_var(self, X, Fmu, Fvar):
        f = lambda SND, ND: self.likelihood._predict_mean_and_var([], SND[0], SND[1])
        return self._broadcast(f, [Fmu, Fvar], [])
