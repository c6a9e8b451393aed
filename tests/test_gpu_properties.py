"""Shape/size property tests, driven by hypothesis: odd N, M not
a multiple of any tile size, D in {1, 2, 8, 16}, K in {1, 3, 8, 16}, S in 1..9.

For every drawn shape the drop-in SMGP ELBO (models.py:69-79), the per-layer
conditionals (models.py:126-144) and predict_y / predict_assign match the float64 oracle at the north_star
tolerance (ELBO 1e-4 relative, fmean / fvar 1e-4 normwise), and the per-layer
launches agree with the layer-batched ones bit for bit.  The examples are
derandomized (a fixed sequence, no example database), so a failure reproduces.
Lengthscales and M are drawn where Kuu + 1e-6 I stays moderately conditioned; the
conditionals' tolerance grows with the conditioning as K3's own test does
(max(1e-4, 10 sqrt(cond(Kuu)) 1.2e-7): float32 L^-1 of a cond-1e6 Kuu is that far
from float64 whatever computes it), the ELBO's stays 1e-4."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from oracle import cpu_ref as R
from tests.helpers import build_model, dev_noise, normwise, to_np

pytestmark = pytest.mark.gpu

_SETTINGS = settings(max_examples=30, deadline=None, derandomize=True, database=None,
                     suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


@st.composite
def shapes(draw, n_min=2, ls_min=0.25):
    D = draw(st.sampled_from([1, 2, 8, 16]))
    K = draw(st.sampled_from([1, 3, 8, 16]))
    N = draw(st.integers(min_value=n_min, max_value=3001))
    m_max = min(N, 24 if D == 1 else (96 if D == 2 else 300))
    M = draw(st.integers(min_value=1, max_value=m_max))
    S = draw(st.integers(min_value=1, max_value=9))
    ls = draw(st.floats(min_value=ls_min, max_value=max(ls_min, 0.5) if D <= 2 else 1.5))
    return N, M, K, D, S, ls


@_SETTINGS
@given(shape=shapes())
def test_elbo_and_conditionals_random_shapes(device, shape):
    N, M, K, D, S, ls = shape
    print("elbo shape (N, M, K, D, S, ls):", shape, flush=True)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=7)
    ref, parts = R.smgp_elbo(X, Y, p, z, u, return_parts=True)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    assert e == pytest.approx(ref, rel=1e-4), (shape, e, ref)
    mu_f, var_f, mu_a, var_a = model.conditionals(Xd)
    for got, name, L in ((mu_f, "mu_f", p.pred), (var_f, "var_f", p.pred), (mu_a, "mu_a", p.assign),
                         (var_a, "var_a", p.assign)):
        cond = np.linalg.cond(R.rbf_Kuu(L["Z"], L["variance"], L["lengthscales"]))
        tol = max(1e-4, 10 * np.sqrt(cond) * 1.2e-7)
        want = parts[name]
        if np.abs(want).max() == 0:
            assert np.abs(to_np(got)).max() < 1e-6, (shape, name)
        else:
            assert normwise(to_np(got).T, want) < tol, (shape, name, cond)
    # predict_y / predict_assign (models.py:38-41, 85-89) on held-out points
    cond = max(np.linalg.cond(R.rbf_Kuu(L["Z"], L["variance"], L["lengthscales"])) for L in (p.pred, p.assign))
    tol = max(1e-4, 10 * np.sqrt(cond) * 1.2e-7)
    Xt = np.random.default_rng(N + M).standard_normal((min(N, 97), D))
    ym, yv = model.predict_y(torch.as_tensor(Xt, dtype=torch.float32, device=device))
    rm, rv = R.predict_y(Xt.astype(np.float32).astype(np.float64), p)
    # normwise, with an absolute floor where the reference itself is negligible (held-out
    # points far from every Z at a short lengthscale: means ~1e-17 in float64)
    close = lambda got, ref: np.linalg.norm(np.asarray(got, np.float64) - ref) <= tol * max(
        np.linalg.norm(ref), 1e-3 * np.sqrt(ref.size))
    assert close(ym, rm), (shape, "predict_y mean")
    assert close(yv, rv), (shape, "predict_y var")
    pa = model.predict_assign(torch.as_tensor(Xt, dtype=torch.float32, device=device))
    assert close(pa, R.predict_assign(Xt.astype(np.float32).astype(np.float64), p)), (shape, "predict_assign")


@_SETTINGS
@given(shape=shapes())
def test_layer_batched_launches_match_per_layer(device, shape):
    """The layer-batched K4 / K5 (and the tril(q_sqrt) batch) against one launch per
    layer: the same conditionals, bit for bit, at every drawn shape."""
    from modulatedgps_amd import models
    N, M, K, D, S, ls = shape
    print("batch shape (N, M, K, D, S, ls):", shape, flush=True)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    batched = [t.clone() for t in model.conditionals(Xd)]
    flags = (models._K4_BATCHED, models._QS_BATCH)
    try:
        models._K4_BATCHED, models._QS_BATCH = False, False
        per_layer = [t.clone() for t in model.conditionals(Xd)]
    finally:
        models._K4_BATCHED, models._QS_BATCH = flags
    for a, b in zip(batched, per_layer):
        assert torch.equal(a, b), shape


@settings(max_examples=24, deadline=None, derandomize=True, database=None,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(shape=shapes(ls_min=0.5), modified=st.booleans())
def test_elbo_and_grad_random_shapes(device, shape, modified):
    """The whole training gradient (SMGP / SMGPModified elbo_and_grad: K6 backward,
    conditional backward, the batched Cholesky / RBF backward, KL) at drawn shapes
    against float64 autograd of oracle/grad_ref.py: every block within max(3e-4,
    4 x float32 autograd's error).  test_elbo_and_grad holds the configured shapes to
    1.5 x; drawn shapes reach degenerate ones (M = 1, S = 1, a few points per expert)
    where the kernel-variance gradients -- near-cancelling sums (1 - |A|^2 + |L^T A|^2
    terms) -- are 1e-3 off float64 in float32 itself, and there the default format's
    22-bit operands (unit roundoff 2^-22, 4 x float32's) show: e.g. (N, M, K, D, S) =
    (130, 1, 3, 1, 1), assign.variance 5.0e-3 against float32's 2.3e-3; (2, 1, 8, 1, 2),
    2.2e-3 against 8.6e-4.  Lengthscales from 0.5: at 0.25 in one dimension most
    points see K(z, x) ~ 0 and the assign layer's gradients through the
    temperature-0.01 Gumbel-softmax near-cancel — (72, 1, 3, 1, 2, 0.25): float32 autograd
    1.8e-2 off on assign.variance, and the HIP path 10x float32 on assign.lengthscales in
    both image formats alike (x6 = f16 there: not an operand-format effect).  (This test
    found the K = 1 row-stride bug of the K6 backward's G, fixed in ops.elbo_terms_backward.)"""
    from tests.test_gpu_training import _check_elbo_and_grad
    N, M, K, D, S, ls = shape
    print("grad shape (N, M, K, D, S, ls), modified:", shape, modified, flush=True)
    _check_elbo_and_grad(device, N, M, K, D, ls, S, modified, factor=4.0)


@_SETTINGS
@given(shape=shapes(), modified=st.booleans(), cut=st.floats(min_value=0.0, max_value=1.0))
def test_multiclass_and_shard_random_shapes(device, shape, modified, cut):
    """At drawn shapes: the MultiClass / RobustMax pred likelihood (SMGP and
    SMGPModified, K classes from the draw, at least 2) against the float64 oracle
    (ELBO 1e-4 relative), and the data-parallel property the multi-GPU path rests on --
    the Gaussian data term of two N-shards (split at a drawn point, Philox keyed by the
    global row via n_offset) sums to the unsharded one (1e-6 relative)."""
    from modulatedgps_amd import ops
    from tests.test_gpu_multiclass import _model, _problem
    N, M, K, D, S, ls = shape
    K = max(K, 2)
    print("mc/shard shape (N, M, K, D, S, ls), modified, cut:", shape, modified, round(cut, 3), flush=True)
    X, Y, p = _problem(N, M, K, D, ls, S)
    a_var = np.linspace(0.3, 0.9, K)[None, :]
    z, u = R.explicit_noise(S, N, K, seed=5)
    ref = R.smgp_modified_elbo(X, Y, p, a_var, z, u) if modified else R.smgp_elbo(X, Y, p, z, u)
    model = _model(p, device, modified, a_var)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    assert e == pytest.approx(ref, rel=1e-4), (shape, e, ref)
    # N-shard invariance of the Gaussian data term (tests/test_gpu_model.py's property at drawn sizes)
    Xg, Yg, pg = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    gm = build_model(pg, device)
    Xgd = torch.as_tensor(Xg, dtype=torch.float32, device=device)
    Ygd = torch.as_tensor(Yg[:, 0], dtype=torch.float32, device=device)
    lv = gm.likelihood.likelihood.variance.reshape(-1)
    full = [t.clone() for t in gm.conditionals(Xgd)]
    tot = float(ops.elbo_terms(*full, Ygd, lv, S, seed=23).cpu())
    c = min(max(int(round(cut * N)), 1), N - 1)
    parts = 0.0
    for lo, hi in ((0, c), (c, N)):
        cs = [t.clone() for t in gm.conditionals(Xgd[lo:hi])]
        parts += float(ops.elbo_terms(*cs, Ygd[lo:hi].contiguous(), lv, S, seed=23, n_offset=lo).cpu())
    assert parts == pytest.approx(tot, rel=1e-6, abs=1e-9), (shape, c, parts, tot)
