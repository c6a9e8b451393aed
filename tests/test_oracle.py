"""CPU tests of the oracle (oracle/cpu_ref.py, oracle/philox.py) against the pins
available for this path: Random123 known-answer vectors, the reference's own
demo-data generator (fixture), closed-form identities of the SMGP ELBO, and the
golden fixtures under tests/golden/ (which pin the oracle against regressions).

Parity status of the oracle itself: unpinned against TF2/GPflow (not
importable here, no reference tests exist); identity-pinned as below."""
import os

import numpy as np
import pytest

from oracle import cpu_ref as R
from oracle import philox

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def _params_from(d):
    layers = {}
    for name in ("pred", "assign"):
        layers[name] = {k: d[f"{name}_{k}"] for k in ("Z", "variance", "lengthscales", "q_mu", "q_sqrt")}
    return R.SMGPParams(layers["pred"], layers["assign"], d["lik_variance"], int(d["num_data"]),
                        int(d["S"]))


# ----------------------------------------------------------------------------- Philox
@pytest.mark.parametrize("ctr,key,expect", [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
])
def test_philox_known_answers(ctr, key, expect):
    """Random123 kat_vectors for philox4x32_10."""
    out = philox.philox4x32_10(np.array(ctr, np.uint32), np.array(key, np.uint32))
    assert [int(x) for x in out] == expect


def test_philox_streams_are_shard_invariant():
    n = np.arange(1000)
    z_full = philox.noise_normal(7, 3, n, 5)
    z_a = philox.noise_normal(7, 3, n[:400], 5)
    z_b = philox.noise_normal(7, 3, n[400:], 5)
    assert np.array_equal(z_full, np.concatenate([z_a, z_b], 1))
    u = philox.noise_uniform(7, 3, n, 5)
    assert u.min() > 0 and u.max() < 1
    assert abs(z_full.mean()) < 0.05 and abs(z_full.std() - 1) < 0.05
    assert abs(u.mean() - 0.5) < 0.02


# ----------------------------------------------------------------------------- data
def test_demo_data_fixture_matches_reference_generator_sums():
    """Bit-stable PCG64 output of utils/dataset_utils.py:100-114 with default_rng(0)
    (values recorded in SURVEY.md §0)."""
    d = _load("demo_tf2_data.npz")
    assert d["Xtrain"].shape == (1500, 1) and d["Ytrain"].shape == (1500, 1)
    assert d["Xtrain"].sum() == pytest.approx(-240.65821112283982, rel=0, abs=1e-9)
    assert d["Ytrain"].sum() == pytest.approx(-1186.726960660836, rel=0, abs=1e-9)
    assert d["Z"].shape == (25, 1) and d["Z_assign"].shape == (25, 1)


# ----------------------------------------------------------------------------- identities
def test_conditional_at_svgp_init_is_prior():
    """q_mu = 0, q_sqrt = I  =>  fmean = 0, fvar = k(x, x) = variance exactly."""
    X, Y, p = R.synthetic_problem(200, 16, 3, 2, 0.7, state="init", S=4)
    L = p.pred
    mu, var = R.svgp_predict_f_dedup(X, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    assert np.abs(mu).max() == 0.0
    np.testing.assert_allclose(var, L["variance"], rtol=1e-12)
    assert R.gauss_kl_white(L["q_mu"], L["q_sqrt"]) == pytest.approx(0.0, abs=1e-12)


def test_faithful_tiled_equals_dedup():
    """The S tiled copies of models.py:35-36 are identical: the S-deduplicated
    evaluation must agree with the faithful one."""
    X, Y, p = R.synthetic_problem(120, 10, 3, 2, 0.5, state="perturbed", S=4)
    z, u = R.explicit_noise(4, 120, 3)
    e1 = R.smgp_elbo(X, Y, p, z, u, faithful=True)
    e2 = R.smgp_elbo(X, Y, p, z, u, faithful=False)
    assert e1 == pytest.approx(e2, rel=1e-12)


def test_single_expert_closed_form():
    """K = 1: W == 1, so ELBO = mean_n(logsumexp_s(ve) - log S) - KL/N = mean(ve) - KL/N."""
    X, Y, p = R.synthetic_problem(150, 12, 1, 2, 0.5, state="perturbed", S=3)
    z, u = R.explicit_noise(3, 150, 1)
    elbo, parts = R.smgp_elbo(X, Y, p, z, u, return_parts=True)
    ve = R.gaussian_var_exp(parts["mu_f"], parts["var_f"], Y, p.lik_variance)[:, 0]
    kl = parts["kl_f"] + parts["kl_a"]
    assert elbo == pytest.approx(ve.mean() - kl / p.num_data, rel=1e-12)


def test_kuf_at_inducing_points_is_kuu_minus_jitter():
    Z = np.random.default_rng(0).standard_normal((9, 3))
    Kuf = R.rbf_K(Z, Z, 0.7, np.array([0.5, 1.0, 2.0]))
    Kuu = R.rbf_Kuu(Z, 0.7, np.array([0.5, 1.0, 2.0]))
    np.testing.assert_allclose(Kuf, Kuu - R.JITTER * np.eye(9), atol=1e-15)


def test_gauss_kl_matches_dense_formula():
    """Whitened KL(N(m, LL^T) || N(0, I)) = 0.5(tr(LL^T) + m^T m - M - log det(LL^T))."""
    rng = np.random.default_rng(3)
    M, K = 7, 2
    q_mu = rng.standard_normal((M, K))
    q_sqrt = np.tril(rng.standard_normal((K, M, M))) + 2 * np.eye(M)
    ref = 0.0
    for k in range(K):
        S = q_sqrt[k] @ q_sqrt[k].T
        ref += 0.5 * (np.trace(S) + q_mu[:, k] @ q_mu[:, k] - M - np.linalg.slogdet(S)[1])
    assert R.gauss_kl_white(q_mu, q_sqrt) == pytest.approx(ref, rel=1e-12)


def test_relaxed_onehot_is_simplex_and_sharp():
    rng = np.random.default_rng(1)
    logits = rng.standard_normal((50, 4))
    u = rng.uniform(size=(50, 4))
    W = R.relaxed_onehot_sample(logits, u)
    np.testing.assert_allclose(W.sum(-1), 1.0, rtol=1e-12)
    assert np.mean(W.max(-1) > 0.99) > 0.8   # tau = 0.01 -> nearly one-hot


def test_tf_legacy_adam_first_step():
    """Step 1: lr_t = lr * sqrt(1-b2)/(1-b1); update = lr_t * g(1-b1) / (sqrt(g^2 (1-b2)) + eps)."""
    th, m, v = R.adam_tf_legacy_step(np.array([1.0]), np.array([0.5]), np.zeros(1), np.zeros(1), 1, 0.1)
    lr_t = 0.1 * np.sqrt(1 - 0.999) / (1 - 0.9)
    expect = 1.0 - lr_t * 0.05 / (np.sqrt(0.25 * 0.001) + 1e-7)
    assert th[0] == pytest.approx(expect, rel=1e-14)


# ----------------------------------------------------------------------------- golden
@pytest.mark.parametrize("case", ["case_demo_init", "case_demo_perturbed", "case_c1"])
def test_golden_fixture_reproduces(case):
    d = _load(case + ".npz")
    p = _params_from(d)
    elbo, parts = R.smgp_elbo(d["X"], d["Y"], p, d["z"], d["u"], return_parts=True)
    assert elbo == pytest.approx(float(d["elbo"]), rel=1e-12)
    np.testing.assert_allclose(parts["var_f"], d["var_f"], rtol=1e-10)
    my, vy = R.predict_y(d["Xtest"], p)
    np.testing.assert_allclose(my, d["predict_y_mean"], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(R.predict_assign(d["Xtest"], p), d["predict_assign"], rtol=1e-10)


def test_golden_c2_reduced_reproduces():
    d = _load("case_c2r.npz")
    gen = {k[4:]: (v.item() if v.ndim == 0 else v) for k, v in d.items() if k.startswith("gen_")}
    gen["state"] = str(gen["state"])
    X, Y, p = R.synthetic_problem(**gen)
    z, u = R.explicit_noise(25, gen["N"], gen["K"], seed=5)
    assert R.smgp_elbo(X, Y, p, z, u) == pytest.approx(float(d["elbo"]), rel=1e-12)


def test_golden_faithful_matches():
    for case in ("case_demo_init", "case_demo_perturbed"):
        d = _load(case + ".npz")
        assert float(d["elbo_faithful"]) == pytest.approx(float(d["elbo"]), rel=1e-12)


@pytest.mark.parametrize("modified", [False, True])
def test_grad_oracle_value_matches_cpu_oracle(modified):
    """oracle/grad_ref.py (torch float64 autograd) evaluates the same ELBO as
    cpu_ref.smgp_elbo / smgp_modified_elbo, so its gradients are the gradients
    of the pinned forward restatement."""
    import torch
    from oracle import grad_ref as G
    X, Y, p = R.synthetic_problem(300, 12, 3, 2, 0.6, state="perturbed", S=4)
    # the grad oracle holds float32-rounded parameters, as the device does
    for L in (p.pred, p.assign):
        for k in ("Z", "q_mu", "q_sqrt"):
            L[k] = np.asarray(L[k]).astype(np.float32).astype(np.float64)
    z, u = R.explicit_noise(4, 300, 3)
    pred, assign, lik = G.params_from_oracle(p)
    a_var = np.array([[0.4, 0.6, 0.8]])
    e = G.elbo(torch.tensor(X), torch.tensor(Y), pred, assign, lik, torch.tensor(z), torch.tensor(u),
               p.num_data, assign_lik_var=torch.tensor(a_var[0]) if modified else None)
    p.lik_variance = lik.detach().numpy().reshape(1, -1)
    for L, T in ((p.pred, pred), (p.assign, assign)):
        L["variance"] = float(T["variance"].detach())
        L["lengthscales"] = T["lengthscales"].detach().numpy()
    ref = R.smgp_modified_elbo(X, Y, p, a_var, z, u) if modified else R.smgp_elbo(X, Y, p, z, u)
    assert float(e) == pytest.approx(ref, rel=1e-10)
    e.backward()
    assert pred["q_sqrt"].grad is not None and torch.isfinite(pred["q_sqrt"].grad).all()


# ----------------------------------------------------------------------------- MultiClass
def _phi(x):
    from scipy.special import erf
    return 0.5 * (1.0 + erf(x / np.sqrt(2.0)))


def test_robustmax_two_class_closed_form(monkeypatch):
    """K = 2: prob_is_largest(y) = (1 - 2e-6) E[Phi((X - mu_o) / s_o)] + 1e-6 with
    X ~ N(mu_y, v_y), i.e. (1 - 2e-6) Phi((mu_y - mu_o) / sqrt(v_y + v_o)) + 1e-6.
    GPflow's 20-point rule meets it to ~5e-7 for comparable variances (it is an
    approximation: up to ~2e-2 when v_y >> v_o); a 150-point rule to 1e-6."""
    rng = np.random.default_rng(0)
    y = rng.integers(0, 2, (200, 1))
    yi = y.reshape(-1)
    o, r = 1 - yi, np.arange(200)
    mu = rng.normal(0, 1.0, (200, 2))
    for lo, hi, tol in ((0.5, 1.5, 2e-6), (0.05, 1.5, 3e-2)):
        var = rng.uniform(lo, hi, (200, 2))
        p = R.robustmax_prob_is_largest(y, mu, var, 2).reshape(-1)
        exact = (1 - 2e-6) * _phi((mu[r, yi] - mu[r, o]) / np.sqrt(var[r, yi] + var[r, o])) + 1e-6
        assert np.max(np.abs(p - exact)) < tol
    x150, w150 = np.polynomial.hermite.hermgauss(150)
    monkeypatch.setattr(R, "GH_X", x150)
    monkeypatch.setattr(R, "GH_W", w150)
    p = R.robustmax_prob_is_largest(y, mu, var, 2).reshape(-1)
    assert np.max(np.abs(p - exact)) < 1e-6


def test_robustmax_class_probabilities_sum_to_one():
    """sum_i P(i is the largest) = 1 up to the squash and the quadrature."""
    rng = np.random.default_rng(1)
    for K in (3, 4, 6):
        mu = rng.normal(0, 1.0, (100, K))
        var = rng.uniform(0.3, 1.0, (100, K))
        tot = sum(R.robustmax_prob_is_largest(np.full((100, 1), i), mu, var, K).reshape(-1) for i in range(K))
        assert np.max(np.abs(tot - 1.0)) < 1e-3   # squash + the 20-point rule


def test_robustmax_limits_and_predictive():
    """Vanishing variances: p -> 1 for the largest latent (minus the squash); an
    out-of-range label selects no class (tf.one_hot -> zero row); the MultiClass
    predictive mean is p (1 - eps) + (1 - p) eps / (K - 1) and sums to one."""
    mu = np.array([[2.0, 0.0, -1.0], [0.0, 3.0, 1.0]])
    var = np.full((2, 3), 1e-12)
    p = R.robustmax_prob_is_largest(np.array([[0], [1]]), mu, var, 3).reshape(-1)
    assert np.allclose(p, (1 - 2e-6) ** 2 + 2e-6 * (1 - 2e-6), atol=1e-9)
    p_out = R.robustmax_prob_is_largest(np.array([[5], [5]]), mu, var, 3).reshape(-1)
    assert np.all(p_out < 1e-5)
    ps, pv = R.multiclass_predict_mean_and_var(mu, np.full((2, 3), 0.3), 3, eps=1e-3)
    assert np.allclose(ps.sum(1), 1.0, atol=1e-4)
    assert np.allclose(pv, ps - ps ** 2)
    ve = R.multiclass_var_exp(mu, var, np.array([[0], [1]]), 3, eps=1e-3)
    assert np.allclose(ve, p * np.log(1 - 1e-3) + (1 - p) * np.log(1e-3 / 2), rtol=1e-12)


@pytest.mark.parametrize("modified", [False, True])
def test_multiclass_grad_oracle_matches_cpu_oracle(modified):
    """grad_ref's differentiable MultiClass var-exp and ELBO equal cpu_ref's."""
    import torch
    from oracle import grad_ref as G
    rng = np.random.default_rng(2)
    mu, var = rng.normal(0, 1, (50, 3)), rng.uniform(0.05, 1.0, (50, 3))
    y = rng.integers(0, 3, (50, 1)).astype(np.float64)
    ref = R.multiclass_var_exp(mu, var, y, 3, eps=1e-3)
    got = G.multiclass_var_exp(torch.tensor(mu), torch.tensor(var), y, 1e-3).numpy()
    assert np.allclose(got, ref, rtol=1e-12, atol=1e-12)
    X, _, p = R.synthetic_problem(300, 12, 3, 2, 0.6, state="perturbed", S=4)
    Y = rng.integers(0, 3, (300, 1)).astype(np.float64)
    for L in (p.pred, p.assign):
        for k in ("Z", "q_mu", "q_sqrt"):
            L[k] = np.asarray(L[k]).astype(np.float32).astype(np.float64)
    p.multiclass_eps = 1e-3
    z, u = R.explicit_noise(4, 300, 3)
    pred, assign, lik = G.params_from_oracle(p)
    a_var = np.array([[0.4, 0.6, 0.8]])
    e = G.elbo(torch.tensor(X), torch.tensor(Y), pred, assign, lik, torch.tensor(z), torch.tensor(u),
               p.num_data, assign_lik_var=torch.tensor(a_var[0]) if modified else None, multiclass_eps=1e-3)
    for L, T in ((p.pred, pred), (p.assign, assign)):
        L["variance"] = float(T["variance"].detach())
        L["lengthscales"] = T["lengthscales"].detach().numpy()
    ref = R.smgp_modified_elbo(X, Y, p, a_var, z, u) if modified else R.smgp_elbo(X, Y, p, z, u)
    assert float(e) == pytest.approx(ref, rel=1e-10)
    # the multiclass pred term ignores W up to sum_k W = 1: it differs from the Gaussian one
    p.multiclass_eps = None
    assert abs(R.smgp_elbo(X, Y, p, z, u) - R.smgp_elbo(X, Y, R.SMGPParams(
        p.pred, p.assign, p.lik_variance, p.num_data, p.S, multiclass_eps=1e-3), z, u)) > 1e-3
