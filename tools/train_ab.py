"""A/B of host-side training-step knobs at c3: interleaved rounds of timed
training steps (elbo_and_grad + TF-legacy Adam) per setting, ms per step.
Usage: python tools/train_ab.py [rounds] [steps]   (settings: backward_streams 1 / 2)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from modulatedgps_amd import config  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    X_np, Y_np, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, num_data=cfg[0])
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    from modulatedgps_amd.training import AdamTF
    opt = AdamTF(model.trainable_parameters(), 1e-3)
    settings = [1, 2]
    res = {s: [] for s in settings}
    for s in settings:   # warm both (workspaces, code objects)
        config.set_backward_streams(s)
        for _ in range(3):
            e, g = model.elbo_and_grad(X, Y)
            opt.step(g)
    torch.cuda.synchronize()
    for r in range(rounds):
        for s in settings:
            config.set_backward_streams(s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                e, g = model.elbo_and_grad(X, Y)
                opt.step(g)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / steps
            res[s].append(ms)
            print(f"round {r} backward_streams={s}: {ms:.3f} ms/step ({1e3 / ms:.2f} steps/s)", flush=True)
    for s in settings:
        print(f"backward_streams={s}: best {min(res[s]):.3f} ms, median {sorted(res[s])[len(res[s]) // 2]:.3f} ms")


if __name__ == "__main__":
    main()
