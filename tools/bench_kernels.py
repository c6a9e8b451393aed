"""Per-kernel micro-benchmark at BASELINE config shapes (HIP events, interleaved
repeats in one process).  Usage: python tools/bench_kernels.py [--config c3] [--reps 5]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402

CFG = {"c2": (8192, 256, 4, 2, 0.15), "c3": (65536, 1024, 8, 8, 1.0), "c5": (262144, 2048, 16, 16, 2.0)}


def timeit(fn, reps, inner=10):
    """Median / min over `reps` of the mean time of `inner` back-to-back calls
    (amortises the host launch latency of short kernels)."""
    ts = []
    for _ in range(reps):
        fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(inner):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / inner)
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="", help="comma-separated subset of the kernels to time")
    a = ap.parse_args()
    N, M, K, D, ls = CFG[a.config]
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, D, device=dev, generator=g)
    Z = X[:M].clone()
    var = torch.tensor([0.5], device=dev)
    lsc = torch.tensor([ls], device=dev)
    q_mu = 0.5 * torch.randn(M, K, device=dev, generator=g)
    q_sqrt = ops.padded(M, M, dev, batch=K)
    q_sqrt.copy_(0.5 * torch.eye(M, device=dev) + torch.tril(0.1 * torch.randn(K, M, M, device=dev, generator=g)))
    out = {}
    _, LinvT, info = ops.kuu_potrf_trtri([Z, Z], [var, var], [lsc, lsc], 1e-6)
    Kuf = ops.rbf_kuf(X, Z, var, lsc)
    A, stats = ops.trsm_stats(LinvT[0], Kuf, q_mu)
    fm, fv = ops.expert_conditional(A, q_sqrt, stats, var)
    Kfr = ops.rbf_kuf_x6(X, Z, var, lsc)
    Tfr = ops.split_upper_x6(LinvT[0])
    Afr, st6 = ops.trsm_stats_x6(Tfr, Kfr, q_mu, M, N)
    Lfr = ops.split_lower_x6(q_sqrt)
    fm6, fv6 = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K)
    # split-f16 forward hand-off (the default forward format)
    Ahr = torch.empty_like(Afr)
    sth = torch.empty_like(st6)
    Lhr = ops.split_lower_x6(q_sqrt, fmt="f16")
    ops.trsm_stats_x6(Tfr, Kfr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var)
    Khr = ops.rbf_kuf_x6(X, Z, var, lsc, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var, in_fmt="f16")
    # backward operands
    A32 = ops.padded(M, N, dev)
    ops.trsm_stats_x6(Tfr, Kfr, q_mu, M, N, Afr=Afr, stats=st6, A=A32)
    G = ops.padded(2 * K, N, dev)
    G.copy_(1e-3 * torch.randn(2 * K, N, device=dev, generator=g))
    Gmu, Gv = G[:K], G[K:]
    P = ops.padded(M, M, dev, batch=K)
    gK = ops.padded(M, N, dev)
    gK.copy_(torch.randn(M, N, device=dev, generator=g))
    gLm = ops.padded(M, M, dev)
    wsg = torch.empty(max(ops._lib.load().mgp_gram_x6_workspace_bytes(M, M, N, K, 2),
                          ops._lib.load().mgp_gram_x6_workspace_bytes(M, M, N, 1, 1)), dtype=torch.uint8, device=dev)
    gbnd = (A32[:, :N].abs().max().reshape(1), A32[:, :N].abs().max().reshape(1), Gv[:, :N].abs().max().reshape(1))
    arows = ops.split_rows_f16(A32, gbnd[0], N=N)
    Lc, LinvTc, _ = ops.kuu_potrf_trtri([Z], [var], [lsc], 1e-6, want_L=True)
    gLc = ops.padded(M, M, dev)
    gLc.copy_(torch.tril(torch.randn(M, M, device=dev, generator=g)))
    cb = ops.conditional_backward_x6(Afr, A32, q_sqrt, q_mu, LinvT[0], Gmu, Gv, M, N)
    wsc = torch.empty(ops.conditional_backward_workspace_bytes(M, N, K), dtype=torch.uint8, device=dev)
    A32h = ops.padded(M, N, dev)   # the f16 chain's training K4: f16 A image + f32 A
    ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, A=A32h, f16_variance=var, in_fmt="f16", cross="f8")
    cbh = ops.conditional_backward_x6(Ahr, A32h, q_sqrt, q_mu, LinvT[0], Gmu, Gv, M, N, fmt="f16")
    Cfr = torch.empty(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=dev)
    colmax = ops.colnorm_max(q_sqrt)
    ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm6, fvar=fv6, fmt="f16", cross="f16",
                              c_out=(Cfr, colmax))
    cimg = (Cfr, colmax, ops.image_bound(Lhr, M, K=K))
    # both layers in one launch (distinct operand copies for the second layer)
    Thr2, Khr2, Ahr2, Lhr2 = Thr.clone(), Khr.clone(), Ahr.clone(), Lhr.clone()
    sth2 = sth.clone()
    fmB, fvB = fm6.clone(), fv6.clone()
    wsx = [torch.empty(ops.expert_x6_workspace_bytes(M, N, K), dtype=torch.uint8, device=dev) for _ in range(2)]
    torch.cuda.synchronize()
    runs = {
        "trsm_f16_pair": lambda: ops.trsm_stats_f16_batch([Thr, Thr2], [Khr, Khr2], [q_mu, q_mu], M, N, [Ahr, Ahr2],
                                                          [sth, sth2], [var, var]),
        "expert_cond_f16_pair": lambda: ops.expert_conditional_f16_batch([Ahr, Ahr2], [Lhr, Lhr2], [sth, sth2],
                                                                         [var, var], M, N, K, [fm6, fmB], [fv6, fvB],
                                                                         wsx),
        "kuu_chol_x2": lambda: ops.kuu_potrf_trtri([Z, Z], [var, var], [lsc, lsc], 1e-6, LinvT=LinvT, info=info),
        "kuu_chol_kuf_x2": lambda: ops.kuu_potrf_trtri([Z, Z], [var, var], [lsc, lsc], 1e-6, LinvT=LinvT, info=info,
                                                       kuf=(X, [Khr, Khr2], "f16")),
        "kuu_chol_x1": lambda: ops.kuu_potrf_trtri([Z], [var], [lsc], 1e-6, LinvT=LinvT[0:1], info=info[0:1]),
        "rbf_kuf": lambda: ops.rbf_kuf(X, Z, var, lsc, out=Kuf),
        "trsm_stats": lambda: ops.trsm_stats(LinvT[0], Kuf, q_mu, A=A, stats=stats),
        "expert_cond": lambda: ops.expert_conditional(A, q_sqrt, stats, var, fmean=fm, fvar=fv),
        "rbf_kuf_x6": lambda: ops.rbf_kuf_x6(X, Z, var, lsc, out=Kfr),
        "split_upper_x6": lambda: ops.split_upper_x6(LinvT[0], out=Tfr),
        "trsm_stats_x6": lambda: ops.trsm_stats_x6(Tfr, Kfr, q_mu, M, N, Afr=Afr, stats=st6),
        "trsm_x6_nostats": lambda: ops._lib.call("mgp_trsm_stats_x6", Tfr.data_ptr(), Tfr.numel(), Kfr.data_ptr(),
                                                 Kfr.numel(), M, N, q_mu.data_ptr(), K, K, Afr.data_ptr(),
                                                 Afr.numel(), None, N, None, N, ops._stream()),
        "split_lower_x6": lambda: ops.split_lower_x6(q_sqrt, out=Lfr),
        "expert_cond_x6": lambda: ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K, fmean=fm6, fvar=fv6),
        "trsm_stats_x6f16": lambda: ops.trsm_stats_x6(Tfr, Kfr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var),
        "rbf_kuf_f16": lambda: ops.rbf_kuf_x6(X, Z, var, lsc, out=Khr, fmt="f16"),
        "split_upper_f16": lambda: ops.split_upper_x6(LinvT[0], out=Thr, fmt="f16"),
        "trsm_stats_f16": lambda: ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var,
                                                    in_fmt="f16", cross="f16"),
        "trsm_stats_f16x8": lambda: ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var,
                                                      in_fmt="f16", cross="f8"),
        "trsm_f16_nostats": lambda: ops._lib.call("mgp_trsm_stats_f16", Thr.data_ptr(), Thr.numel(), Khr.data_ptr(),
                                                  Khr.numel(), M, N, q_mu.data_ptr(), K, K, var.data_ptr(),
                                                  Ahr.data_ptr(), Ahr.numel(), None, N, None, N, ops._stream()),
        "split_lower_f16": lambda: ops.split_lower_x6(q_sqrt, out=Lhr, fmt="f16"),
        "expert_cond_f16": lambda: ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm6, fvar=fv6,
                                                             fmt="f16", cross="f16"),
        "expert_cond_f16x8": lambda: ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm6, fvar=fv6,
                                                               fmt="f16", cross="f8"),
        "gram_x6_P": lambda: ops.gram_x6(A32, A32, Gv, mode=2, N=N, out=P, workspace=wsg),
        "gram_x6_Lm": lambda: ops.gram_x6(gK, A32, None, mode=1, N=N, out=gLm, workspace=wsg),
        "gram_f16_P": lambda: ops.gram_x6(A32, A32, Gv, mode=2, N=N, out=P, workspace=wsg, bounds=gbnd),
        "gram_f16_rows_P": lambda: ops.gram_x6(A32, A32, Gv, mode=2, N=N, out=P, workspace=wsg, bounds=gbnd,
                                               x_rows=arows),
        "rbf_bwd": lambda: ops.rbf_backward(X, Z, var, lsc, gK),
        "chol_bwd": lambda: ops.chol_backward(Lc[0], LinvTc[0], gLc),
        "cond_bwd_x6": lambda: ops.conditional_backward_x6(Afr, A32, q_sqrt, q_mu, LinvT[0], Gmu, Gv, M, N,
                                                           out=cb, workspace=wsc),
        "cond_bwd_f16": lambda: ops.conditional_backward_x6(Ahr, A32h, q_sqrt, q_mu, LinvT[0], Gmu, Gv, M, N,
                                                            out=cbh, workspace=wsc, fmt="f16", cross="f16"),
        "cond_bwd_f16c": lambda: ops.conditional_backward_x6(Ahr, A32h, q_sqrt, q_mu, LinvT[0], Gmu, Gv, M, N,
                                                             out=cbh, workspace=wsc, fmt="f16", cross="f16",
                                                             c_images=cimg),
        "cond_bwd_f16x8": lambda: ops.conditional_backward_x6(Ahr, A32h, q_sqrt, q_mu, LinvT[0], Gmu, Gv, M, N,
                                                              out=cbh, workspace=wsc, fmt="f16", cross="f8"),
    }
    if a.only:
        runs = {k: v for k, v in runs.items() if k in a.only.split(",")}
    for _ in range(2):
        for f in runs.values():
            f()
    torch.cuda.synchronize()
    for name, f in runs.items():
        med, mn = timeit(f, a.reps)
        out[name] = {"median_ms": med, "min_ms": mn}
    if "expert_cond" in out:
        out["expert_cond"]["tflops"] = K * M * M * N / (out["expert_cond"]["median_ms"] * 1e-3) / 1e12
    if "expert_cond_x6" in out:
        out["expert_cond_x6"]["tflops"] = K * M * M * N / (out["expert_cond_x6"]["median_ms"] * 1e-3) / 1e12
    if "expert_cond_f16_pair" in out:
        out["expert_cond_f16_pair"]["tflops"] = 2 * K * M * M * N / (out["expert_cond_f16_pair"]["median_ms"] * 1e-3) / 1e12
    if "trsm_f16_pair" in out:
        out["trsm_f16_pair"]["tflops"] = 2 * M * M * N / (out["trsm_f16_pair"]["median_ms"] * 1e-3) / 1e12
    for name in ("expert_cond_f16", "expert_cond_f16x8"):
        if name in out:
            out[name]["tflops"] = K * M * M * N / (out[name]["median_ms"] * 1e-3) / 1e12
    for name in ("trsm_stats_x6", "trsm_stats_x6f16", "trsm_stats_f16", "trsm_stats_f16x8"):
        if name in out:
            out[name]["tflops"] = M * M * N / (out[name]["median_ms"] * 1e-3) / 1e12
    for name, fl in (("gram_x6_P", K * M * M * N), ("gram_x6_Lm", M * M * N), ("gram_f16_P", K * M * M * N),
                     ("gram_f16_rows_P", K * M * M * N),
                     ("cond_bwd_x6", (2 * K + 1) * M * M * N), ("cond_bwd_f16", (2 * K + 1) * M * M * N),
                     ("cond_bwd_f16c", (K + 1) * M * M * N)):
        if name in out:
            out[name]["tflops"] = fl / (out[name]["median_ms"] * 1e-3) / 1e12
    if "rbf_bwd" in out:
        out["rbf_bwd"]["GBps"] = 4 * M * N / (out["rbf_bwd"]["median_ms"] * 1e-3) / 1e9
    if "rbf_kuf_x6" in out:
        out["rbf_kuf_x6"]["GBps"] = (4 * (N * D + M * D) + 6 * M * N) / (out["rbf_kuf_x6"]["median_ms"] * 1e-3) / 1e9
    if "rbf_kuf_f16" in out:
        out["rbf_kuf_f16"]["GBps"] = (4 * (N * D + M * D) + 4 * M * N) / (out["rbf_kuf_f16"]["median_ms"] * 1e-3) / 1e9
    if "trsm_stats" in out:
        out["trsm_stats"]["tflops"] = M * M * N / (out["trsm_stats"]["median_ms"] * 1e-3) / 1e12
    if "rbf_kuf" in out:
        out["rbf_kuf"]["GBps"] = 4 * (N * D + M * D + M * N) / (out["rbf_kuf"]["median_ms"] * 1e-3) / 1e9
    print(json.dumps({"config": a.config, "env": {k: v for k, v in os.environ.items() if k.startswith("MGP_")}, **out}))


if __name__ == "__main__":
    main()
