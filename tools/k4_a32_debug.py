"""Debug: K4's f32 A from the 16x16 and 32x32 kernels at a small shape; prints where they
differ and, for each differing s16 value, where it sits in the s32 result."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402


def main():
    N, M, K, D = 512, 256, 4, 2
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, D, device=dev, generator=g)
    Z = X[:M].clone()
    var, ls = torch.tensor([0.5], device=dev), torch.tensor([1.0], device=dev)
    q_mu = 0.5 * torch.randn(M, K, device=dev, generator=g)
    _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
    Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    res = {}
    for shape in ("32", "16"):
        os.environ["MGP_K4_SHAPE"] = shape
        A32 = ops.padded(M, N, dev, zero=True)
        ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, A=A32, f16_variance=var, in_fmt="f16")
        torch.cuda.synchronize()
        res[shape] = A32[:, :N].double().cpu().numpy()
    a, b = res["32"], res["16"]
    ref = (LinvT[0].double().cpu().numpy()[:M, :M].T) @ ops_kuf(X, Z, var, ls, dev)
    print("normwise 32 vs ref", np.linalg.norm(a - ref) / np.linalg.norm(ref))
    print("normwise 16 vs ref", np.linalg.norm(b - ref) / np.linalg.norm(ref))
    bad = np.argwhere(np.abs(a - b) > 1e-4 * np.abs(a).max())
    print("n bad", len(bad), "of", a.size)
    for r, c in bad[:24]:
        j = np.argwhere(np.abs(a - b[r, c]) < 1e-6 * max(abs(b[r, c]), 1e-30))
        print((int(r), int(c)), "s32", a[r, c], "s16", b[r, c], "s16 value found in s32 at", j[:3].tolist())


def ops_kuf(X, Z, var, ls, dev):
    Kuf = ops.rbf_kuf(X, Z, var, ls)
    torch.cuda.synchronize()
    return Kuf[:, :X.shape[0]].double().cpu().numpy()


if __name__ == "__main__":
    main()
