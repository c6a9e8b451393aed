"""Would one K4 launch over both layers beat two?  Times the split-f16 K4
(mgp_trsm_stats_f16) at N = 65536 twice back to back against one launch at
N = 131072 (the same per-workgroup work, twice the workgroups), c3 shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    M, K, D = 1024, 8, 8
    g = torch.Generator(device=dev).manual_seed(0)
    var = torch.tensor([0.5], device=dev)
    ls = torch.tensor([1.0], device=dev)
    Z = torch.randn(M, D, device=dev, generator=g)
    _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
    q_mu = 0.5 * torch.randn(M, K, device=dev, generator=g)
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    res = {}
    for N in (65536, 131072):
        X = torch.randn(N, D, device=dev, generator=g)
        Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
        out = [ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, f16_variance=var, in_fmt="f16", cross="f16")
               for _ in range(2)]
        reps = 2 if N == 65536 else 1

        def run():
            for i in range(reps):
                ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=out[i][0], stats=out[i][1], f16_variance=var,
                                  in_fmt="f16", cross="f16")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / 20)
        res[f"{reps} x N={N}"] = sorted(ts)
    for k, v in res.items():
        print(f"{k}: median {v[2]:.1f} us, min {v[0]:.1f} us per pair of layers")


if __name__ == "__main__":
    main()
