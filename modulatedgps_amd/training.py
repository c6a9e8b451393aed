"""Optimiser of the training step: TF 2.10 Keras-legacy Adam on the unconstrained
variables (utils/training_utils.py:6,10), one HIP kernel
launch for all parameter blocks (mgp_adam_step_set, csrc/train.hip; one launch per
block when there are more than 16).

Positive parameters (GPflow positive() = softplus) keep an unconstrained shadow
u = softplus^-1(theta) on the device; Adam updates u and the kernel refreshes
theta = softplus(u) in the same launch.  Free parameters are updated in place.
q_sqrt is updated as a dense [K*M, M] block: its gradient is zero above the
diagonal, so the upper triangle stays zero (the same trajectory as Adam on the
packed FillTriangular vector, since Adam is elementwise)."""
import torch

from . import ops

_ADAM_SET = True   # False: one mgp_adam_step launch per block (A/B probes only)


def _as2d(t):
    if t.dim() == 1:
        return t.view(1, -1)
    if t.dim() == 3:
        return t.flatten(0, 1)
    return t


class AdamTF:
    """tf.optimizers.Adam(lr) (beta1 0.9, beta2 0.999, epsilon 1e-7) over
    model.trainable_parameters()."""

    def __init__(self, params, lr, beta1=0.9, beta2=0.999, epsilon=1e-7):
        self.params = list(params)
        self.lr, self.beta1, self.beta2, self.eps = float(lr), float(beta1), float(beta2), float(epsilon)
        self.t = 0
        self.state = {}
        for name, theta, kind in self.params:
            v = _as2d(theta)
            st = {"m1": torch.zeros(v.shape, dtype=torch.float32, device=theta.device),
                  "m2": torch.zeros(v.shape, dtype=torch.float32, device=theta.device), "u": None}
            if kind == "positive":   # u = softplus^-1(theta) (parameter transform, set once)
                th = theta.detach().double()
                st["u"] = torch.where(th > 20, th, torch.log(torch.expm1(th))).float().reshape(v.shape).contiguous()
            self.state[name] = st

    def step(self, grads):
        """Apply one step from the ELBO gradients (dict name -> tensor)."""
        self.t += 1
        if _ADAM_SET and len(self.params) <= 16:
            if getattr(self, "_set", None) is None:
                self._set = ops.AdamSet([(_as2d(theta), self.state[name]["m1"], self.state[name]["m2"],
                                          self.state[name]["u"]) for name, theta, _ in self.params])
            self._set.step([_as2d(grads[name]) for name, _, _ in self.params], self.t, self.lr, beta1=self.beta1,
                           beta2=self.beta2, eps=self.eps, grad_sign=-1.0)
            return
        for name, theta, kind in self.params:
            st = self.state[name]
            ops.adam_step(_as2d(theta), _as2d(grads[name]), st["m1"], st["m2"], self.t, self.lr, u=st["u"],
                          beta1=self.beta1, beta2=self.beta2, eps=self.eps, grad_sign=-1.0)
