"""ELBO step at c3 under environment switches read per call (A/B in one process,
interleaved rounds).  Prints ms/step per setting and the ELBO of each.
Usage: python tools/env_ab_probe.py '{"base": {}, "k1first": {"MGP_K1_FIRST": "1"}}'"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {"base": {}, "k1first": {"MGP_K1_FIRST": "1"}}
    keys = sorted({k for v in variants.values() for k in v})
    cfg = bench.CONFIGS["c3"]
    dev = torch.device("cuda", 0)
    X, Y, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, cfg[0])
    Xd = torch.as_tensor(X, device=dev)
    Yd = torch.as_tensor(Y, device=dev)
    times = {n: [] for n in variants}
    elbo = {}
    for rnd in range(int(os.environ.get("ROUNDS", "6"))):
        for name, env in variants.items():
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(5):
                model._build_likelihood(Xd, Yd, seed=11)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(40):
                e = model._build_likelihood(Xd, Yd, seed=11)
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / 40 * 1e3)
            elbo[name] = float(e.cpu())
        print("round", rnd, {n: round(t[-1], 4) for n, t in times.items()}, flush=True)
    print(json.dumps({n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)), "elbo": elbo[n]}
                      for n, t in times.items()}))


if __name__ == "__main__":
    main()
