"""Run the c3 training step (elbo_and_grad + TF-legacy Adam) `n` times after a
warmup, for a rocprofv3 --kernel-trace --stats profile of the step's kernels.
Usage: python tools/train_steps.py [n]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    X_np, Y_np, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, num_data=cfg[0])
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    from modulatedgps_amd.training import AdamTF
    opt = AdamTF(model.trainable_parameters(), 1e-3)
    for _ in range(3 + n):
        e, g = model.elbo_and_grad(X, Y)
        opt.step(g)
    torch.cuda.synchronize()
    print("elbo", float(e.item()))


if __name__ == "__main__":
    main()
