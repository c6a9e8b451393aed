"""ELBO step at c3 under environment switches read per call (A/B in one process,
interleaved rounds).  Prints ms/step per setting and the ELBO of each.  TRAIN=1: the
step is elbo_and_grad (ELBO + full gradient; no optimizer update, so every variant
sees the same parameters) and the gradients' normwise difference to the first
variant is printed too.  CONFIG=c5 for BASELINE config 5.
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
    cfg = bench.CONFIGS[os.environ.get("CONFIG", "c3")]
    train = os.environ.get("TRAIN") == "1"
    dev = torch.device("cuda", 0)
    X, Y, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, cfg[0])
    Xd = torch.as_tensor(X, device=dev)
    Yd = torch.as_tensor(Y, device=dev)
    times = {n: [] for n in variants}
    elbo, grads = {}, {}
    nsteps = int(os.environ.get("STEPS", "40" if not train else "10"))

    def step():
        if train:
            return model.elbo_and_grad(Xd, Yd, seed=11)
        return model._build_likelihood(Xd, Yd, seed=11), None
    for rnd in range(int(os.environ.get("ROUNDS", "6"))):
        for name, env in variants.items():
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(nsteps):
                e, g = step()
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / nsteps * 1e3)
            elbo[name] = float(e.detach().cpu())
            if g is not None and name not in grads:
                grads[name] = {k: v.detach().double().clone() for k, v in g.items()}
        print("round", rnd, {n: round(t[-1], 4) for n, t in times.items()}, flush=True)
    out = {n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t)), "elbo": elbo[n]}
           for n, t in times.items()}
    if grads:
        first = next(iter(grads))
        for n in grads:
            out[n]["grad_normwise_vs_" + first] = max(
                float((grads[n][k] - grads[first][k]).norm() / grads[first][k].norm().clamp_min(1e-300))
                for k in grads[first])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
