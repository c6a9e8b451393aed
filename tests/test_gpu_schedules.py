"""Every step schedule (config.STEP_SCHEDULES) computes the same bits.

The schedules only move the Cholesky-independent work of a step (K1, the tril(q_sqrt)
images, the KL) between the main and the side stream, and the k1a_* ones run the
layers' K4 / K5 per layer instead of in one launch each (the batch entries are
bit-identical to the per-layer ones).  So, for a fixed Philox key, the ELBO of
_build_likelihood (models.py:69-79) and the ELBO and every gradient block of
elbo_and_grad (utils/training_utils.py:10) must be bit-identical to the default
schedule's.  Shapes: equal M for both layers (the batched K3 / K4 / K5 path),
ragged N."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from tests.helpers import build_model

pytestmark = pytest.mark.gpu


def _run(device, sched, train):
    from modulatedgps_amd import config
    old = config.step_schedule()
    config.set_step_schedule(sched)
    try:
        X, Y, p = R.synthetic_problem(3001, 128, 4, 3, 0.8, state="perturbed", S=6)
        model = build_model(p, device)
        Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
        if train:
            e, g = model.elbo_and_grad(Xd, Y, seed=1234)
            return e.clone(), {k: v.clone() for k, v in g.items()}
        return model._build_likelihood(Xd, Y, seed=1234), None
    finally:
        config.set_step_schedule(old)


@pytest.mark.parametrize("train", [False, True], ids=["forward", "training"])
def test_step_schedules_bit_identical(device, train):
    from modulatedgps_amd import config
    ref_e, ref_g = _run(device, config.STEP_SCHEDULES[0], train)
    assert np.isfinite(float(ref_e.cpu()))
    for sched in config.STEP_SCHEDULES[1:]:
        e, g = _run(device, sched, train)
        assert torch.equal(e, ref_e), (sched, float(e), float(ref_e))
        if train:
            assert sorted(g) == sorted(ref_g)
            for k in ref_g:
                assert torch.equal(g[k], ref_g[k]), (sched, k)
