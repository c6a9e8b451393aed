"""Timed c3 training steps (elbo_and_grad + TF-legacy Adam) of the library in
MGP_HIP_LIB (default: the in-tree one), for A/B runs of kernel variants in
separate processes: prints ms per step for `rounds` blocks of `steps` steps.
Usage: python tools/train_ab.py [rounds] [steps] [label]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    label = sys.argv[3] if len(sys.argv) > 3 else os.environ.get("MGP_HIP_LIB", "in-tree")
    if "colmaxmain" in sys.argv[4:]:   # colnorm_max on the main stream before K5 (before round 4's move)
        from modulatedgps_amd import models
        models._COLMAX_SIDE = False
    if "k4single" in sys.argv[4:]:   # one K4 launch per layer (the round-4 default before the batch)
        from modulatedgps_amd import models
        models._K4_BATCHED = False
    if "tailper" in sys.argv[4:]:   # Cholesky / RBF backward per layer (before round 5's batch)
        from modulatedgps_amd import models
        models._TAIL_BATCH = False
    if "fill" in sys.argv[4:]:   # zero-filled gZ / g_ls + accumulate (before the overwrite mode)
        from modulatedgps_amd import models
        models._RBF_NO_FILL = False
    if "noprep" in sys.argv[4:]:   # the C-images backward's q_sqrt launches inside it (before the prep)
        from modulatedgps_amd import models
        models._COND_PREP = False
    if "notb" in sys.argv[4:]:   # max |LinvT| reduced inside the backward (before the K3 bound hand-over)
        from modulatedgps_amd import models
        models._T_BOUND = False
    if "adamper" in sys.argv[4:]:   # one Adam launch per parameter block (before round 5's set)
        from modulatedgps_amd import training
        training._ADAM_SET = False
    dev = torch.device("cuda", 0)
    cfg = bench.CONFIGS["c3"]
    X_np, Y_np, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, num_data=cfg[0])
    X = torch.from_numpy(X_np).to(dev)
    Y = torch.from_numpy(Y_np).to(dev)
    from modulatedgps_amd.training import AdamTF
    opt = AdamTF(model.trainable_parameters(), 1e-3)
    for _ in range(3):
        e, g = model.elbo_and_grad(X, Y)
        opt.step(g)
    torch.cuda.synchronize()
    res = []
    for r in range(rounds):
        t0 = time.perf_counter()
        for _ in range(steps):
            e, g = model.elbo_and_grad(X, Y)
            opt.step(g)
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t0) * 1e3 / steps)
    print(f"{label}: " + " ".join(f"{m:.3f}" for m in res) + f" ms/step; best {min(res):.3f} "
          f"({1e3 / min(res):.2f} steps/s)", flush=True)


if __name__ == "__main__":
    main()
