"""Shared test helpers: build device models from oracle parameter sets."""
import os

import numpy as np
import torch

from oracle import cpu_ref as R

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def params_from_golden(d):
    layers = {}
    for name in ("pred", "assign"):
        layers[name] = {k: d[f"{name}_{k}"] for k in ("Z", "variance", "lengthscales", "q_mu", "q_sqrt")}
    return R.SMGPParams(layers["pred"], layers["assign"], d["lik_variance"], int(d["num_data"]),
                        int(d["S"]))


def build_model(p, device, seed=0):
    """SMGP on the device from an oracle SMGPParams (float64 -> float32)."""
    from modulatedgps_amd.kernels import SquaredExponential
    from modulatedgps_amd.likelihoods import GaussianModified
    from modulatedgps_amd.models import SMGP, SVGPModified

    K = p.lik_variance.shape[1]
    lik = GaussianModified(variance=p.lik_variance, device=device)
    layers = []
    for L in (p.pred, p.assign):
        kern = SquaredExponential(variance=L["variance"], lengthscales=L["lengthscales"], device=device)
        layer = SVGPModified(kern, lik, L["Z"], num_latent_gps=K, whiten=True, device=device)
        layer.set_variational(L["q_mu"], L["q_sqrt"])
        layers.append(layer)
    return SMGP(lik, layers[0], layers[1], K=K, num_samples=p.S, num_data=p.num_data, seed=seed)


def normwise(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


def to_np(t):
    if isinstance(t, np.ndarray):  # the public predict_* return host arrays
        return np.asarray(t, np.float64)
    return t.detach().double().cpu().numpy()


def dev_noise(z, u, device):
    return (torch.as_tensor(z, dtype=torch.float32, device=device),
            torch.as_tensor(u, dtype=torch.float32, device=device))


def decode_cols_image(img, M, N):
    """Split-bf16 column image (modulatedgps_amd/csrc/split3.hip layout
    [nb][mk][plane][lane][8]) -> float64 [M, N] = hi + mid + lo."""
    Mp, Np = -(-M // 128) * 128, -(-N // 256) * 256
    nb, nmk = Np // 32, Mp // 16
    u16 = img.detach().cpu().numpy().view(np.uint16)[: nb * nmk * 3 * 64 * 8].reshape(nb, nmk, 3, 64, 8)
    f = (u16.astype(np.uint32) << 16).view(np.float32).astype(np.float64).sum(axis=2)  # [nb][mk][64][8]
    lane, j = np.arange(64), np.arange(8)
    kp = (j[None, :] & 3) + 8 * (j[None, :] >> 2) + 4 * (lane[:, None] >> 5)          # [64][8]
    rows = 16 * np.arange(nmk)[None, :, None, None] + kp[None, None]
    cols = 32 * np.arange(nb)[:, None, None, None] + (lane & 31)[None, None, :, None]
    out = np.zeros((Mp, Np))
    out[np.broadcast_to(rows, f.shape), np.broadcast_to(cols, f.shape)] = f
    return out[:M, :N]


def decode_cols_f16(img, M, N, bound):
    """Split-f16 column image (planes 0 / 1 = fp16 hi / lo of x 2^e, e = 13 - ilogb(bound);
    modulatedgps_amd/csrc/mgp_common.hpp) -> float64 [M, N] = (hi + lo) 2^-e."""
    Mp, Np = -(-M // 128) * 128, -(-N // 256) * 256
    nb, nmk = Np // 32, Mp // 16
    u = img.detach().cpu().numpy().view(np.float16)[: nb * nmk * 3 * 64 * 8].reshape(nb, nmk, 3, 64, 8)
    e = 13 - int(np.floor(np.log2(bound)))
    f = (u[:, :, 0].astype(np.float64) + u[:, :, 1].astype(np.float64)) * 2.0 ** -e
    lane, j = np.arange(64), np.arange(8)
    kp = (j[None, :] & 3) + 8 * (j[None, :] >> 2) + 4 * (lane[:, None] >> 5)
    rows = 16 * np.arange(nmk)[None, :, None, None] + kp[None, None]
    cols = 32 * np.arange(nb)[:, None, None, None] + (lane & 31)[None, None, :, None]
    out = np.zeros((Mp, Np))
    out[np.broadcast_to(rows, f.shape), np.broadcast_to(cols, f.shape)] = f
    return out[:M, :N]
