"""K6 backward at a given lane build vs the shipped build: runs ops.elbo_terms_backward on fixed
random inputs (explicit noise and in-kernel Philox) for a list of small shapes and saves G and the
likelihood-variance gradients to gpurun_out/k6b_<label>.npz (compare two labels with --compare).
    python tools/k6b_lanes_diff.py LABEL          (library from MGP_HIP_LIB or in-tree)
    python tools/k6b_lanes_diff.py --compare A B"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(9, 3, 1, False), (9, 3, 1, True), (9, 3, 5, False), (37, 8, 25, False), (1000, 3, 25, False)]


def run(label):
    import torch
    from modulatedgps_amd import ops
    dev = torch.device("cuda", 0)
    out = {}
    for (N, K, S, mod) in SHAPES:
        g = torch.Generator(device="cpu").manual_seed(N * 100 + K * 10 + S)
        mu_f = ops.padded(K, N, dev); mu_f.copy_(torch.randn(K, N, generator=g))
        var_f = ops.padded(K, N, dev); var_f.copy_(torch.rand(K, N, generator=g) + 0.1)
        mu_a = ops.padded(K, N, dev); mu_a.copy_(torch.randn(K, N, generator=g))
        var_a = ops.padded(K, N, dev); var_a.copy_(torch.rand(K, N, generator=g) * 0.1)
        Y = torch.randn(N, generator=g).to(dev)
        lv = (torch.rand(K, generator=g) + 0.5).to(dev)
        lva = (torch.rand(K, generator=g) + 0.5).to(dev) if mod else None
        z = torch.randn(S, N, K, generator=g).to(dev)
        u = torch.rand(S, N, K, generator=g).clamp(1e-6, 1 - 1e-6).to(dev)
        for tag, noise in (("explicit", (z, u)), ("philox", None)):
            G, glv, glva = ops.elbo_terms_backward(mu_f, var_f, mu_a, var_a, Y, lv, S, noise=noise, seed=7,
                                                   assign_lik_var=lva, scale=1.0 / N)
            torch.cuda.synchronize()
            key = f"{N}_{K}_{S}_{int(mod)}_{tag}"
            out[key + "_G"] = G.cpu().numpy()
            out[key + "_glv"] = glv.cpu().numpy()
            if glva is not None:
                out[key + "_glva"] = glva.cpu().numpy()
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez(f"gpurun_out/k6b_{label}.npz", **out)


def compare(a, b):
    A, B = np.load(f"gpurun_out/k6b_{a}.npz"), np.load(f"gpurun_out/k6b_{b}.npz")
    for k in A.files:
        x, y = A[k].astype(np.float64), B[k].astype(np.float64)
        d = np.abs(x - y).max() / max(np.abs(y).max(), 1e-30)
        rows = "" if x.ndim < 3 else " rows(max rel by [4,K]): " + str(
            np.round(np.abs(x - y).max(axis=-1) / np.maximum(np.abs(y).max(axis=-1), 1e-30), 6).tolist())
        print(f"{k:32s} max rel diff {d:.3e}{rows if d > 1e-5 else ''}")


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
