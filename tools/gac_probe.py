"""The training backward's gA from the C_k images on 16x16x32 MFMAs (grad_a_c16_kernel,
the default) against grad_a_c_kernel (MGP_GAC_SHAPE=32) at c3, one process: the
conditional backward's outputs compared (normwise) and its time per call (HIP events,
interleaved rounds).  Usage: python tools/gac_probe.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402


def main():
    N, M, K, D = 65536, 1024, 8, 8
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, D, device=dev, generator=g)
    Z = X[:M].clone()
    var, ls = torch.tensor([0.5], device=dev), torch.tensor([1.0], device=dev)
    q_mu = 0.5 * torch.randn(M, K, device=dev, generator=g)
    q_sqrt = ops.padded(M, M, dev, batch=K)
    q_sqrt.copy_(0.5 * torch.eye(M, device=dev) + torch.tril(0.1 * torch.randn(K, M, M, device=dev, generator=g)))
    _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
    Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    A32 = ops.padded(M, N, dev)
    Ahr, sth = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, A=A32, f16_variance=var, in_fmt="f16")
    Lhr = ops.split_lower_x6(q_sqrt, fmt="f16")
    Cfr = torch.empty(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=dev)
    colmax = ops.colnorm_max(q_sqrt)
    ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16", c_out=(Cfr, colmax))
    G = ops.padded(2 * K, N, dev)
    G.copy_(1e-3 * torch.randn(2 * K, N, device=dev, generator=g))
    cimg = (Cfr, colmax, ops.image_bound(Lhr, M, K=K))
    wsc = torch.empty(ops.conditional_backward_workspace_bytes(M, N, K), dtype=torch.uint8, device=dev)
    variants = {"gac32": "32", "gac16": "16"}

    def run():
        return ops.conditional_backward_x6(Ahr, A32, q_sqrt, q_mu, LinvT[0], G[:K], G[K:], M, N, workspace=wsc,
                                           fmt="f16", cross="f16", c_images=cimg)

    out = {}
    for name, shape in variants.items():
        os.environ["MGP_GAC_SHAPE"] = shape
        r = run()
        torch.cuda.synchronize()
        out[name] = {k: v.double().clone() for k, v in r.items() if torch.is_tensor(v)}
    errs = {k: float((out["gac16"][k] - out["gac32"][k]).norm() / out["gac32"][k].norm().clamp_min(1e-300))
            for k in out["gac32"]}
    print(errs, flush=True)
    times = {n: [] for n in variants}
    for rnd in range(int(os.environ.get("ROUNDS", "5"))):
        for name, shape in variants.items():
            os.environ["MGP_GAC_SHAPE"] = shape
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 5)
        print("round", rnd, {n: round(t[-1], 4) for n, t in times.items()}, flush=True)
    print(json.dumps({"normwise_16_vs_32": errs,
                      **{n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for n, t in times.items()}}))


if __name__ == "__main__":
    main()
