"""K5 (split-f16) shape variants in one process at c3: the 32x32x16 kernel
(MGP_K5_SHAPE=32) against the 16x16x32 kernel (the default), interleaved rounds, HIP events, random operands;
checks that both give the same fvar (normwise).  Usage: python tools/k5_probe.py"""
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
    Ahr, sth = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, f16_variance=var, in_fmt="f16")
    Lhr = ops.split_lower_x6(q_sqrt, fmt="f16")
    res = {}
    variants = {"s32": "32", "s16": "16"}
    for name, shape in variants.items():
        os.environ["MGP_K5_SHAPE"] = shape
        fm, fv = ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16")
        torch.cuda.synchronize()
        res[name] = fv[:, :N].double().clone()
    err = float((res["s16"] - res["s32"]).norm() / res["s32"].norm())
    # training K5 (writes the C_k images): both shapes, the images compared as decoded f16 planes
    Cfr = {n: torch.empty(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=dev) for n in variants}
    colmax = ops.colnorm_max(q_sqrt)
    for name, shape in variants.items():
        os.environ["MGP_K5_SHAPE"] = shape
        Cfr[name].zero_()
        ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16", c_out=(Cfr[name], colmax))
    torch.cuda.synchronize()
    h = {n: Cfr[n].view(torch.float16).float() for n in variants}
    cerr = float((h["s16"] - h["s32"]).norm() / h["s32"].norm())
    # conditional backward from each shape's C images (the backward kernels themselves are shape-independent)
    A32 = ops.padded(M, N, dev)
    ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, A=A32, f16_variance=var, in_fmt="f16")
    G = ops.padded(2 * K, N, dev)
    G.copy_(1e-3 * torch.randn(2 * K, N, device=dev, generator=g))
    cimg = (Cfr["s16"], colmax, ops.image_bound(Lhr, M, K=K))
    wsc = torch.empty(ops.conditional_backward_workspace_bytes(M, N, K), dtype=torch.uint8, device=dev)
    cb = {}
    for name, shape in variants.items():
        os.environ["MGP_K5_SHAPE"] = shape
        cb[name] = ops.conditional_backward_x6(Ahr, A32, q_sqrt, q_mu, LinvT[0], G[:K], G[K:], M, N, workspace=wsc,
                                               fmt="f16", cross="f16", c_images=cimg)
        torch.cuda.synchronize()
        cb[name] = {k: v.double().clone() for k, v in cb[name].items() if torch.is_tensor(v)}
    gerr = float((cb["s16"]["g_Kuf"] - cb["s32"]["g_Kuf"]).norm() / cb["s32"]["g_Kuf"].norm())
    times = {n: [] for n in variants}
    times.update({n + "_cout": [] for n in variants})
    times.update({n + "_cbwd": [] for n in variants})
    fm, fv = ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16")
    for _ in range(int(os.environ.get("ROUNDS", "6"))):
        for name, shape in variants.items():
            os.environ["MGP_K5_SHAPE"] = shape
            for _ in range(3):
                ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm, fvar=fv, fmt="f16", cross="f16")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm, fvar=fv, fmt="f16", cross="f16")
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20)
            e0.record()
            for _ in range(10):
                ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm, fvar=fv, fmt="f16", cross="f16",
                                          c_out=(Cfr[name], colmax))
            e1.record()
            torch.cuda.synchronize()
            times[name + "_cout"].append(e0.elapsed_time(e1) / 10)
            e0.record()
            for _ in range(5):
                ops.conditional_backward_x6(Ahr, A32, q_sqrt, q_mu, LinvT[0], G[:K], G[K:], M, N, workspace=wsc,
                                            fmt="f16", cross="f16", c_images=cimg)
            e1.record()
            torch.cuda.synchronize()
            times[name + "_cbwd"].append(e0.elapsed_time(e1) / 5)
    print(json.dumps({"fvar_normwise_16_vs_32": err, "cimg_normwise_16_vs_32": cerr, "gKuf_normwise_16_vs_32": gerr,
                      **{n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for n, t in times.items()}}))


if __name__ == "__main__":
    main()
