"""reparameterize (MixtureGPs/utils.py:8-36) and print_summary (the
gpflow.utilities.print_summary the demos call, demos/demo_tf2.py:49,58).

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


def print_summary(model, fmt=None):
    """Parameter table of an SMGP / SGP model (name, transform, shape, dtype, value),
    the content of gpflow.utilities.print_summary(model) for the demos; returns
    the text as well as printing it."""
    rows = []
    params = model.trainable_parameters() if hasattr(model, "trainable_parameters") else []
    for name, t, kind in params:
        v = t.detach().float().cpu()
        if v.numel() <= 4:
            val = "[" + ", ".join(f"{x:.6g}" for x in v.reshape(-1).tolist()) + "]"
        else:
            val = f"mean {v.mean().item():.4g}, min {v.min().item():.4g}, max {v.max().item():.4g}"
        rows.append((f"{type(model).__name__}.{name}", "Softplus" if kind == "positive" else
                     ("FillTriangular" if name.endswith("q_sqrt") else "Identity"),
                     str(tuple(t.shape)), str(t.dtype).replace("torch.", ""), val))
    head = ("name", "transform", "shape", "dtype", "value")
    w = [max(len(r[i]) for r in rows + [head]) for i in range(5)]
    line = lambda r: "| " + " | ".join(c.ljust(w[i]) for i, c in enumerate(r)) + " |"
    text = "\n".join([line(head), "|" + "|".join("-" * (x + 2) for x in w) + "|"] + [line(r) for r in rows])
    print(text)
    return text
