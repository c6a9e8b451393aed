"""Debug: per-block errors (HIP / float32 autograd, vs float64) of one drawn gradient
case in the f16 and x6 formats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import config  # noqa: E402
import tests.test_gpu_training as T  # noqa: E402

dev = torch.device("cuda", 0)
case = (72, 1, 3, 1, 0.25, 2, False)
for fmt in ("f16", "x6"):
    config.set_expert_format(fmt)
    try:
        T._check_elbo_and_grad(dev, *case, factor=1e9)
    except AssertionError as e:
        print("assert", e)
    print(fmt, "done", flush=True)
