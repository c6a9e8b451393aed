"""reparameterize (MixtureGPs/utils.py:8-36).

The diagonal path ``mean + z * sqrt(var + jitter)`` (utils.py:26-27) is the one
the SMGP uses; inside the ELBO it is fused into mgp_elbo_terms.  The reference's
full_cov=True branch calls a non-existent ``tf.cholesky`` (utils.py:30) and is
unreachable from the models; here it is implemented with the same semantics
(var [S, N, N, D]) for completeness.
"""
import torch

from .config import default_jitter


def reparameterize(mean, var, z, full_cov=False):
    if var is None:
        return mean
    if not full_cov:
        return mean + z * (var + default_jitter()) ** 0.5
    S, N, D = mean.shape
    mean = mean.permute(0, 2, 1)                      # SND -> SDN
    var = var.permute(0, 3, 1, 2)                     # SNND -> SDNN
    eye = default_jitter() * torch.eye(N, dtype=var.dtype, device=var.device)[None, None]
    chol = torch.linalg.cholesky(var + eye)
    z_res = z.permute(0, 2, 1)[..., None]             # SND -> SDN1
    f = mean + (chol @ z_res)[..., 0]
    return f.permute(0, 2, 1)
