"""The reference's method-level surface on the MI355X kernels, against the float64
oracle (1e-4 normwise / relative, the north_star tolerance):

  SVGPModified.posterior(precompute_cache)              models.py:148-160
    -> IndependentPosteriorSingleOutputModified
       ._conditional_fused / fused_predict_f            models.py:126-144
  SMGP.W_dist(Xt) -> RelaxedOneHotCategorical.sample    models.py:55-61,73-74
  SMGP.E_log_p_Y(Xt, Y, W)                              models.py:63-67
  SMGPModified.E_log_p_Y                                models.py:112-123
  model.trainable_variables                             utils/training_utils.py:10

and the composition the reference's _build_likelihood makes of them
(models.py:69-79) equal to the fused K6 path with the same Philox key."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from tests.helpers import build_model, dev_noise, load_golden, normwise, params_from_golden, to_np

pytestmark = pytest.mark.gpu


def _golden(device, case="case_demo_perturbed"):
    d = load_golden(case + ".npz")
    p = params_from_golden(d)
    return d, p, build_model(p, device)


@pytest.mark.parametrize("case", ["case_demo_perturbed", "case_c1"])
def test_posterior_conditional_fused(device, case):
    from modulatedgps_amd.models import IndependentPosteriorSingleOutputModified, PrecomputeCacheType
    d, p, model = _golden(device, case)
    S = 4
    X = d["X"]
    Xt = R.integrate(X, S)                                                 # [S, N, D] tiled (models.py:35-36)
    L = p.pred
    mu_ref, var_ref = R.svgp_predict_f(Xt, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    post = model.pred_layer.posterior(PrecomputeCacheType.NOCACHE)
    assert isinstance(post, IndependentPosteriorSingleOutputModified)
    Xd = torch.as_tensor(Xt, dtype=torch.float32, device=device)
    fm, fv = post._conditional_fused(Xd, full_cov=False, full_output_cov=False)
    assert tuple(fm.shape) == tuple(mu_ref.shape) and tuple(fv.shape) == tuple(var_ref.shape)
    assert normwise(to_np(fm), mu_ref) < 1e-4
    assert normwise(to_np(fv), var_ref) < 1e-4
    fm2, fv2 = post.fused_predict_f(Xd)
    assert torch.equal(fm2, fm) and torch.equal(fv2, fv)
    # predict_f goes through the same plugin (GPflow SVGP.predict_f -> posterior(NOCACHE))
    fm3, fv3 = model.pred_layer.predict_f(Xd)
    assert normwise(to_np(fm3), to_np(fm)) < 1e-7 and normwise(to_np(fv3), to_np(fv)) < 1e-7
    # tiling is recognised without a device sync: an expand() view (integrate's output)
    # and a host array are computed once (stride 0), a materialised device copy row by row
    lay = model.pred_layer
    Xe = torch.as_tensor(X, dtype=torch.float32, device=device)[None].expand(S, *X.shape)
    assert lay._marginals_kn(Xe)[4] == 0 and lay._marginals_kn(Xt)[4] == 0
    assert lay._marginals_kn(Xd)[4] == X.shape[0]
    fm4, fv4 = post._conditional_fused(Xe)
    assert normwise(to_np(fm4), to_np(fm)) < 1e-6 and normwise(to_np(fv4), to_np(fv)) < 1e-6
    # explicit opt-in for a materialised tiled copy (tf.tile's result): computed once,
    # the same bits as the stride-0 view; tiled=False computes every row
    assert lay._marginals_kn(Xd, tiled=True)[4] == 0 and lay._marginals_kn(Xe, tiled=False)[4] == X.shape[0]
    fm5, fv5 = post._conditional_fused(Xd, tiled=True)
    assert torch.equal(fm5, fm4) and torch.equal(fv5, fv4)
    # distinct inputs per sample (no tiling): one conditional over all S * N rows
    rng = np.random.default_rng(3)
    Xr = X[None] + 0.1 * rng.standard_normal((S,) + X.shape)
    mu_r, var_r = R.svgp_predict_f(Xr, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    fm, fv = post._conditional_fused(torch.as_tensor(Xr, dtype=torch.float32, device=device))
    assert normwise(to_np(fm), mu_r) < 1e-4 and normwise(to_np(fv), var_r) < 1e-4


def test_w_dist_and_sample(device):
    d, p, model = _golden(device)
    S, (N, K) = int(d["S"]), d["mu_a"].shape
    Xt = torch.as_tensor(R.integrate(d["X"], S), dtype=torch.float32, device=device)
    z, u = dev_noise(d["z"], d["u"], device)
    wd = model.W_dist(Xt, noise_z=z)
    assert wd.temperature == pytest.approx(1e-2) and tuple(wd.logits.shape) == (S * N, K)
    logits_ref = R.reparameterize(d["mu_a"][None], d["var_a"][None], d["z"]).reshape(S * N, K)
    assert normwise(to_np(wd.logits), logits_ref) < 1e-4
    W = wd.sample(1, noise_u=u)
    assert tuple(W.shape) == (1, S * N, K)
    # the sampler alone, on the device's logits: the Gumbel-softmax at tau = 0.01
    W_ref = R.relaxed_onehot_sample(to_np(wd.logits), d["u"].reshape(S * N, K))
    assert normwise(to_np(W[0]), W_ref) < 1e-4
    assert np.allclose(to_np(W[0]).sum(1), 1.0, atol=1e-5)
    # Philox mode: fresh draws per sample, rows still on the simplex
    W2 = model.W_dist(Xt, seed=7).sample(3)
    assert tuple(W2.shape) == (3, S * N, K) and not torch.equal(W2[0], W2[1])
    assert np.allclose(to_np(W2).sum(-1), 1.0, atol=1e-5)
    # TFP sample shapes: sample() -> [S * N, K], sample((2, 2)) -> [2, 2, S * N, K]
    wd3 = model.W_dist(Xt, seed=11)
    W3 = wd3.sample()
    assert tuple(W3.shape) == (S * N, K)
    assert tuple(wd3.sample((2, 2)).shape) == (2, 2, S * N, K)
    # an empty sample (TFP: shape [0, S * N, K]) draws nothing: the model's key stream
    # does not advance
    draws = model._draws
    assert tuple(wd3.sample(0).shape) == (0, S * N, K) and tuple(wd3.sample((0, 3)).shape) == (0, 3, S * N, K)
    assert model._draws == draws
    # explicit normals and no seed: every sample() call draws a fresh key
    wd4 = model.W_dist(Xt, noise_z=z)
    assert not torch.equal(wd4.sample(), wd4.sample())


def test_e_log_p_y(device):
    d, p, model = _golden(device)
    S, (N, K) = int(d["S"]), d["mu_a"].shape
    W = R.assignment_weights(d["mu_a"][None], d["var_a"][None], d["z"], d["u"])          # [S, N, K]
    ref = R.e_log_p_y(np.broadcast_to(d["mu_f"], (S, N, K)), np.broadcast_to(d["var_f"], (S, N, K)), d["Y"],
                      p.lik_variance, W, S)
    Xt = torch.as_tensor(R.integrate(d["X"], S), dtype=torch.float32, device=device)
    out = model.E_log_p_Y(Xt, d["Y"], torch.as_tensor(W, dtype=torch.float32, device=device))
    assert tuple(out.shape) == (N,)
    assert normwise(to_np(out), ref) < 1e-4
    # the reference's _build_likelihood composed from the methods (models.py:69-79)
    kl = float(model.pred_layer.prior_kl().cpu()) + float(model.assign_layer.prior_kl().cpu())
    elbo = float(out.mean().cpu()) - kl / p.num_data
    assert elbo == pytest.approx(float(d["elbo"]), rel=1e-4)


@pytest.mark.parametrize("case", ["case_demo_perturbed", "case_c1"])
def test_methods_compose_to_build_likelihood(device, case):
    """W_dist(Xt, seed) -> sample(1) -> E_log_p_Y draws K6's own noise streams, so
    the reference's composition equals the fused kernel with the same key."""
    d, p, model = _golden(device, case)
    S, N = int(d["S"]), d["X"].shape[0]
    Xd = torch.as_tensor(d["X"], dtype=torch.float32, device=device)
    Xt = Xd[None].expand(S, *Xd.shape)
    seed = 1234567
    W = model.W_dist(Xt, seed=seed).sample(1)[0].reshape(S, N, model.K)
    L = model.E_log_p_Y(Xt, d["Y"], W).double().mean()
    kl = model.pred_layer.prior_kl().double() + model.assign_layer.prior_kl().double()
    composed = float((L - kl / p.num_data).cpu())
    fused = float(model._build_likelihood(Xd, d["Y"], seed=seed).cpu())
    assert composed == pytest.approx(fused, rel=2e-6, abs=1e-6)


@pytest.mark.parametrize("multiclass", [False, True])
def test_modified_e_log_p_y(device, multiclass):
    from modulatedgps_amd.kernels import SquaredExponential
    from modulatedgps_amd.likelihoods import GaussianModified, MultiClass, RobustMax
    from modulatedgps_amd.models import SMGPModified, SVGPModified
    N, M, K, D, S = 700, 30, 3, 2, 9
    X, Y, p = R.synthetic_problem(N, M, K, D, 0.8, state="perturbed", S=S)
    eps = 1e-3
    if multiclass:
        Y = np.random.default_rng(2).integers(0, K, (N, 1)).astype(np.float64)
        p.multiclass_eps = eps
        lik = MultiClass(num_classes=K, invlink=RobustMax(K, epsilon=eps, device=device), device=device)
    else:
        lik = GaussianModified(variance=p.lik_variance, device=device)
    a_var = np.linspace(0.3, 0.9, K)[None, :]
    layers = []
    for Lp in (p.pred, p.assign):
        kern = SquaredExponential(variance=Lp["variance"], lengthscales=Lp["lengthscales"], device=device)
        layer = SVGPModified(kern, lik, Lp["Z"], num_latent_gps=K, whiten=True, device=device)
        layer.set_variational(Lp["q_mu"], Lp["q_sqrt"])
        layers.append(layer)
    model = SMGPModified(lik, GaussianModified(variance=a_var, device=device), layers[0], layers[1], K=K,
                         num_samples=S, num_data=N)
    z, u = R.explicit_noise(S, N, K, seed=5)
    mu_a, var_a = R.svgp_predict_f_dedup(X, *(p.assign[k] for k in ("Z", "variance", "lengthscales", "q_mu",
                                                                     "q_sqrt")))
    mu_f, var_f = R.svgp_predict_f_dedup(X, *(p.pred[k] for k in ("Z", "variance", "lengthscales", "q_mu",
                                                                   "q_sqrt")))
    W = R.assignment_weights(mu_a[None], var_a[None], z, u)
    ve_a = R.gaussian_var_exp(mu_a[None], var_a[None], Y[None], a_var)
    ve_f = R.pred_var_exp(mu_f[None], var_f[None], Y, p, S)
    ref = (R._logsumexp0(np.sum(ve_a * W, 2) - np.log(S)) + R._logsumexp0(np.sum(ve_f * W, 2) - np.log(S)))
    Xt = torch.as_tensor(R.integrate(X, S), dtype=torch.float32, device=device)
    out = model.E_log_p_Y(Xt, Y, torch.as_tensor(W, dtype=torch.float32, device=device))
    assert normwise(to_np(out), ref) < 1e-4
    # composition == the fused MOD kernel with the same key
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    Wk = model.W_dist(Xd[None].expand(S, N, D), seed=99).sample(1)[0].reshape(S, N, K)
    L = model.E_log_p_Y(Xd[None].expand(S, N, D), Y, Wk).double().mean()
    kl = model.pred_layer.prior_kl().double() + model.assign_layer.prior_kl().double()
    fused = float(model._build_likelihood(Xd, Y, seed=99).cpu())
    assert float((L - kl / N).cpu()) == pytest.approx(fused, rel=2e-6, abs=1e-6)


def test_trainable_variables(device):
    _, _, model = _golden(device)
    tv = model.trainable_variables
    tp = model.trainable_parameters()
    assert len(tv) == len(tp) and all(a is b for a, (_, b, _) in zip(tv, tp))
    names = [n for n, _, _ in tp]
    assert names[:5] == ["pred.Z", "pred.q_mu", "pred.q_sqrt", "pred.variance", "pred.lengthscales"]
    assert "lik_variance" in names
    assert model.pred_layer.trainable_variables[0] is model.pred_layer.Z
    # the gradient dict of the training step covers every trainable variable
    d = load_golden("case_demo_perturbed.npz")
    _, grads = model.elbo_and_grad(torch.as_tensor(d["X"], dtype=torch.float32, device=device), d["Y"], seed=3)
    for n, t, _ in tp:
        assert grads[n].numel() == t.numel(), n


def test_unconstrained_variables_and_gradients(device):
    """GPflow's trainable_variables are the unconstrained values (softplus^-1 for the
    positive ones); unconstrained_variables / elbo_and_grad(unconstrained=True) /
    assign_unconstrained give a custom loop those semantics: the gradient is the
    constrained one times softplus'(u) = 1 - exp(-theta), the free blocks unchanged,
    and a plain gradient-ascent step on u raises the ELBO."""
    d, p, model = _golden(device)
    X = torch.as_tensor(d["X"], dtype=torch.float32, device=device)
    u = model.unconstrained_variables()
    tp = model.trainable_parameters()
    for n, t, kind in tp:
        back = torch.nn.functional.softplus(u[n].double()).float() if kind == "positive" else u[n]
        assert torch.allclose(back, t, rtol=1e-6, atol=1e-7), n
    e0 = float(model._build_likelihood(X, d["Y"], seed=5).cpu())
    _, g = model.elbo_and_grad(X, d["Y"], seed=5)
    g = {k: v.clone() for k, v in g.items()}
    _, gu = model.elbo_and_grad(X, d["Y"], seed=5, unconstrained=True)
    for n, t, kind in tp:
        ref = g[n] * (-torch.expm1(-t.double())).float() if kind == "positive" else g[n]
        assert normwise(to_np(gu[n]), to_np(ref)) < 1e-6, n
    gnorm = float(torch.sqrt(sum((gu[n].double() ** 2).sum() for n, _, _ in tp)).cpu())
    lr = 1e-3 / gnorm   # a step of length 1e-3 along the gradient
    model.assign_unconstrained({n: u[n] + lr * gu[n] for n, _, _ in tp})
    e1 = float(model._build_likelihood(X, d["Y"], seed=5).cpu())
    assert e1 > e0
    model.assign_unconstrained(u)   # back to the start
    assert float(model._build_likelihood(X, d["Y"], seed=5).cpu()) == pytest.approx(e0, rel=1e-6)
