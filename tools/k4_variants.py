"""K4 (split-f16 in and out) on 16x16x32 MFMAs (trsm_stats16_kernel, the default) against
the 32x32x16 kernel (MGP_K4_SHAPE=32) in one process at c3: outputs compared (A's image
planes decoded, the stats, the f32 A of the training variant), interleaved timing rounds
with HIP events.  Usage: python tools/k4_variants.py"""
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
    _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
    Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    variants = {"s32": "32", "s16": "16"}
    out = {}
    for name, shape in variants.items():
        os.environ["MGP_K4_SHAPE"] = shape
        A32 = ops.padded(M, N, dev)
        Ahr, sth = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, A=A32, f16_variance=var, in_fmt="f16")
        torch.cuda.synchronize()
        out[name] = (Ahr.clone(), sth.clone(), A32[:, :N].clone())
    a, b = out["s32"], out["s16"]
    nb = ops.x6_cols_bytes(M, N) - 256   # planes 0, 1 of every 3 KiB fragment (plane 2 unused in f16)
    img_a = a[0][:nb].view(torch.float16).view(-1, 3, 512)[:, :2].float()
    img_b = b[0][:nb].view(torch.float16).view(-1, 3, 512)[:, :2].float()
    res = {"image_normwise": float((img_b - img_a).norm() / img_a.norm()),
           "image_bit_equal": bool(torch.equal(img_a, img_b)),
           "stats_normwise": float((b[1].double() - a[1].double()).norm() / a[1].double().norm()),
           "a32_normwise": float((b[2].double() - a[2].double()).norm() / a[2].double().norm())}
    print(res, flush=True)
    times = {n: [] for n in variants}
    Ahr, sth = out["s16"][0], out["s16"][1]
    for rnd in range(int(os.environ.get("ROUNDS", "6"))):
        for name, shape in variants.items():
            os.environ["MGP_K4_SHAPE"] = shape
            for _ in range(3):
                ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var, in_fmt="f16")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=sth, f16_variance=var, in_fmt="f16")
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20)
        print("round", rnd, {n: round(t[-1], 4) for n, t in times.items()}, flush=True)
    print(json.dumps({**res, **{n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))}
                                for n, t in times.items()}}))


if __name__ == "__main__":
    main()
