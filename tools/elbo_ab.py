"""Timed c3 ELBO steps of the library in MGP_HIP_LIB (default: the in-tree one),
for A/B runs of kernel variants in separate processes: ms per step for `rounds`
blocks of `steps` steps, and the ELBO at a fixed Philox key (bit-identity check).
Usage: python tools/elbo_ab.py [rounds] [steps] [label]   (MGP_AB_CONFIG=c4r: another bench config)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    label = sys.argv[3] if len(sys.argv) > 3 else os.environ.get("MGP_HIP_LIB", "in-tree")
    if "k4single" in sys.argv[4:]:   # one K4 launch per layer (the round-4 default before the batch)
        from modulatedgps_amd import models
        models._K4_BATCHED = False
    if "qsper" in sys.argv[4:]:   # the tril(q_sqrt) images and KL per layer (before round 5's batch)
        from modulatedgps_amd import models
        models._QS_BATCH = False
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS[os.environ.get("MGP_AB_CONFIG", "c3")]   # e.g. c4r: c4's per-rank shape
    X_np, Y_np, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, num_data=cfg[0])
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    for _ in range(5):
        model._build_likelihood(X, Y)
    e = float(model._build_likelihood(X, Y, seed=777).item())
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        for _ in range(steps):
            model._build_likelihood(X, Y)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) * 1e3 / steps)
    print(f"{label}: " + " ".join(f"{m:.4f}" for m in res) + f" ms/step; best {min(res):.4f} "
          f"({1e3 / min(res):.1f} ELBO/s); elbo(key 777) {e!r}", flush=True)


if __name__ == "__main__":
    main()
