"""K4 (trsm_stats16_kernel, split-f16) with the epilogue splitting each accumulator
once (default) or once per use (MGP_K4_SPLIT_ONCE=0): A image and stats compared
bit for bit, then both timed in interleaved rounds (HIP events, c3 shapes).
Usage: python tools/k4_once_probe.py"""
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
    var, lsc = torch.tensor([0.5], device=dev), torch.tensor([1.0], device=dev)
    q_mu = 0.5 * torch.randn(M, K, device=dev, generator=g)
    _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [lsc], 1e-6)
    Khr = ops.rbf_kuf_x6(X, Z, var, lsc, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    outs = {}
    for name, v in (("twice", "0"), ("once", "1")):
        os.environ["MGP_K4_SPLIT_ONCE"] = v
        Afr, st = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, f16_variance=var, in_fmt="f16", cross="f16")
        torch.cuda.synchronize()
        outs[name] = (Afr.clone(), st.clone())
    same = {"image_equal": bool(torch.equal(outs["once"][0], outs["twice"][0])),
            "stats_equal": bool(torch.equal(outs["once"][1], outs["twice"][1]))}
    print(json.dumps(same), flush=True)
    Afr, st = outs["once"]
    times = {"twice": [], "once": []}
    for _ in range(8):
        for name, v in (("twice", "0"), ("once", "1")):
            os.environ["MGP_K4_SPLIT_ONCE"] = v
            for _ in range(3):
                ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Afr, stats=st, f16_variance=var, in_fmt="f16", cross="f16")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Afr, stats=st, f16_variance=var, in_fmt="f16", cross="f16")
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20 * 1e3)
    print(json.dumps({n: {"median_us": float(np.median(t)), "min_us": float(np.min(t))} for n, t in times.items()}))
    if not (same["image_equal"] and same["stats_equal"]):
        sys.exit(1)


if __name__ == "__main__":
    main()
