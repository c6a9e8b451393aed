"""K3 variants in one process (interleaved rounds): the per-step launches with one tile
per workgroup (chol_step, MGP_CHOL_PAIR=0), with two tiles of a row per 512-thread
workgroup (chol_step_pair, the default) and the persistent launch, c3 shapes (two layers, M = 1024), plus the
largest difference of each variant's L / L^-T to the first.  Usage: python tools/chol_probe.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402


def main():
    M = int(os.environ.get("PROBE_M", "1024"))
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    Z = torch.randn(M, 8, device=dev, generator=g)
    var, ls = torch.tensor([0.5], device=dev), torch.tensor([1.0], device=dev)
    variants = [("tiles", {"MGP_CHOL_PERSIST": "0", "MGP_CHOL_PAIR": "0"}),
                ("pairs", {"MGP_CHOL_PERSIST": "0", "MGP_CHOL_PAIR": "1"}),
                ("persist_w48", {"MGP_CHOL_PERSIST": "1", "MGP_CHOL_WORKERS": "48"})]
    outs = {}
    for name, env in variants:
        os.environ.update(env)
        L, LinvT, info = ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6, want_L=True)
        torch.cuda.synchronize()
        outs[name] = (L.clone(), LinvT.clone(), info.clone())
    ref = outs["tiles"]
    check = {n: {"info": o[2].tolist(), "dL": float((o[0] - ref[0]).abs().max()),
                 "dLinvT": float((o[1] - ref[1]).abs().max())} for n, o in outs.items()}
    print(json.dumps({"check": check}), flush=True)
    times = {n: [] for n, _ in variants}
    for _ in range(5):
        for name, env in variants:
            os.environ.update(env)
            for _ in range(2):
                ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6, LinvT=LinvT)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6, LinvT=LinvT)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / 10)
    print(json.dumps({n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for n, t in times.items()}),
          flush=True)


if __name__ == "__main__":
    main()
