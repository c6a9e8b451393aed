"""Debug: per-block gradient errors of elbo_and_grad against float64 autograd at tiny
shapes (hypothesis found pred.Z wrong at N=2, M=1, K=1, D=1, S=1, ls=0.5)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cpu_ref as R  # noqa: E402
from tests.helpers import build_model, dev_noise, normwise  # noqa: E402
from tests.test_gpu_training import _dense, _oracle  # noqa: E402
from modulatedgps_amd import models  # noqa: E402

dev = torch.device("cuda", 0)
for (N, M, K, D, S, ls) in [(2, 1, 1, 1, 1, 0.5), (2, 1, 1, 1, 1, 0.25), (3, 1, 1, 1, 1, 0.5), (8, 1, 1, 1, 1, 0.5),
                            (8, 2, 1, 1, 1, 0.5), (64, 1, 3, 2, 2, 0.5), (2, 2, 1, 1, 1, 0.5)]:
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    e_ref, g_ref = _oracle(X, Y, p, z, u, None)
    for tail in (True, False):
        models._TAIL_BATCH = tail
        model = build_model(p, dev)
        e, grads = model.elbo_and_grad(torch.as_tensor(X, dtype=torch.float32, device=dev), Y, noise=dev_noise(z, u, dev))
        errs = {}
        for n, _, _ in model.trainable_parameters():
            got = _dense(n, grads[n], M)
            ref = g_ref[n].reshape(got.shape)
            errs[n] = normwise(got, ref)
        bad = {k: f"{v:.1e}" for k, v in errs.items() if v > 3e-4}
        print((N, M, K, D, S, ls), "tail_batch" if tail else "per_layer", "elbo", float(e), e_ref, "bad:", bad, flush=True)
        if bad:
            for k in bad:
                print("   ", k, "got", _dense(k, grads[k], M).ravel()[:6], "ref", g_ref[k].ravel()[:6])
