"""Forward K5 (split-f16) launch variants selected by environment switches, in one
process at c3: interleaved rounds timed with HIP events on random operands, and the
fvar of every variant compared with the first (normwise).
Usage: python tools/k5_variants.py '{"base": {}, "kpair": {"MGP_K5_KPAIR": "1"}}'"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402


def main():
    variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {"base": {}, "kpair": {"MGP_K5_KPAIR": "1"}}
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
    keys = sorted({k for v in variants.values() for k in v})

    def use(name):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update(variants[name])

    out = {}
    for name in variants:
        use(name)
        fm, fv = ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16")
        torch.cuda.synchronize()
        out[name] = (fm[:, :N].double().clone(), fv[:, :N].double().clone())
    first = next(iter(variants))
    errs = {n: {"fvar": float((out[n][1] - out[first][1]).norm() / out[first][1].norm()),
                "fmean": float((out[n][0] - out[first][0]).norm() / out[first][0].norm())} for n in variants}
    times = {n: [] for n in variants}
    fm, fv = ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16")
    for rnd in range(int(os.environ.get("ROUNDS", "6"))):
        for name in variants:
            use(name)
            for _ in range(3):
                ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm, fvar=fv, fmt="f16", cross="f16")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmean=fm, fvar=fv, fmt="f16", cross="f16")
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 20)
        print("round", rnd, {n: round(t[-1], 4) for n, t in times.items()}, flush=True)
    print(json.dumps({"normwise_vs_" + first: errs,
                      **{n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for n, t in times.items()}}))


if __name__ == "__main__":
    main()
