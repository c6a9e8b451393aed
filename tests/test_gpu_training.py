"""GPU parity of the training step (utils/training_utils.py:4-28 run_adam):
the full ELBO gradient assembled by SMGP.elbo_and_grad (K6 backward -> conditional
backward -> Cholesky backward -> RBF backward -> KL) against float64 autograd of
oracle/grad_ref.py at the same explicit noise, and the TF-legacy Adam kernel
against cpu_ref.adam_tf_legacy_step.

Tolerance of the end-to-end gradient (normwise per parameter block, float32
kernels vs float64 autograd): max(3e-4, 1.5 x the error of float32 torch
autograd of the same oracle graph, measured in the test).  The Z / lengthscale
/ variance gradients are sums of large opposing Kuf and Kuu contributions
through an ill-conditioned Cholesky (jitter 1e-6) and, for the assignment
layer, pass the Gumbel-softmax at temperature 0.01, so no fixed float32
tolerance fits every configuration; the criterion asks the HIP path to be as
accurate as a float32 evaluation of the reference's own graph, with the floor for
the blocks whose float32 errors are noise.

Measured at BASELINE config 3 in full (test_elbo_and_grad_c3_full, split-f16, round 6
after the K1 split fix; HIP / float32 autograd, normwise vs float64; tests/
diag_grad_stages.py, profiles/r06f_grad_stages_c3_fixed.json): pred.Z 9.1e-7 / 2.9e-5,
pred.q_mu 7.7e-7 / 3.9e-6, pred.q_sqrt 1.1e-6 / 7.5e-7, pred.lengthscales 5.5e-7 /
2.4e-6, pred.variance 1.5e-7 / 7.5e-8, assign.Z 1.1e-5 / 1.5e-5, assign.q_mu 5.1e-6 /
5.3e-6, assign.q_sqrt 8.9e-7 / 8.5e-7, assign.variance 3.6e-5 / 2.4e-5,
assign.lengthscales 2.1e-5 / 6.6e-6, lik_variance 1.7e-7 / 1.0e-7.  Every block is
within 1.5x of float32 autograd or below it except assign.lengthscales (3.2x),
pred.variance and lik_variance (2x and 1.6x, both ~1e-7).  The lengthscale gradient of
the assignment layer is a sum over all M x N entries of g_Kuf dKuf/dl that cancels
internally: with the float64 G the stage diagnostic finds g_Kuf within 5.3e-7 of
float64 (float32 autograd: 1.1e-6) and the RBF backward itself within 5e-9, yet those
5.3e-7 move the lengthscale gradient by 5.9e-5 where float32 autograd's 1.1e-6 move it
by 1.1e-6 -- float32 autograd's g_Kuf error (a backward-stable triangular solve) is
nearly orthogonal to dKuf/dl, the explicit L^-T product's is not.  Before the K1 fix
(round 5) the assignment blocks were 4-12x worse than float32 autograd (Z 6.5e-5,
lengthscales 6.8e-5, q_mu 3.2e-5, q_sqrt 4.7e-6): the f16 Kuf image at variance 0.1."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from oracle import grad_ref as GR
from tests.helpers import build_model, dev_noise, normwise, to_np

pytestmark = pytest.mark.gpu

FLOOR = 3e-4


def _model(p, device, a_var):
    base = build_model(p, device)
    if a_var is None:
        return base
    from modulatedgps_amd.likelihoods import GaussianModified
    from modulatedgps_amd.models import SMGPModified
    K = p.lik_variance.shape[1]
    return SMGPModified(base.likelihood.likelihood, GaussianModified(variance=a_var, device=device),
                        base.pred_layer, base.assign_layer, K=K, num_samples=p.S, num_data=p.num_data)


def _oracle(X, Y, p, z, u, a_var, dtype=torch.float64):
    pred, assign, lik = GR.params_from_oracle(p)
    leaf = lambda t: t.detach().to(dtype).requires_grad_(True)
    pred = {k: leaf(v) for k, v in pred.items()}
    assign = {k: leaf(v) for k, v in assign.items()}
    lik = leaf(lik)
    f64 = lambda a: torch.tensor(np.asarray(a, np.float32)).to(dtype)
    av = None
    if a_var is not None:
        av = leaf(torch.tensor(np.asarray(a_var, np.float32).reshape(-1)))
    e = GR.elbo(f64(X), f64(Y), pred, assign, lik, f64(z), f64(u), p.num_data, assign_lik_var=av)
    e.backward()
    g = {"lik_variance": lik.grad.double().numpy()}
    if av is not None:
        g["assign_lik_variance"] = av.grad.double().numpy()
    for name, L in (("pred", pred), ("assign", assign)):
        for k in GR.LAYER_KEYS:
            gk = L[k].grad.double().numpy()
            if k == "q_sqrt":
                gk = np.tril(gk)
            g[name + "." + k] = gk
    return float(e.detach()), g


def _dense(name, t, M):
    a = to_np(t)
    return a.reshape(-1) if name.endswith(("variance", "lengthscales")) else a


@pytest.mark.parametrize("N,M,K,D,ls,S,modified", [(1000, 25, 3, 1, 0.5, 25, False),
                                                    (2049, 64, 4, 2, 0.8, 7, False),
                                                    (1000, 25, 3, 1, 0.5, 25, True),
                                                    (4096, 130, 3, 3, 1.0, 5, False),
                                                    (2048, 2048, 16, 16, 2.0, 3, False)])   # config-5 shapes
@pytest.mark.parametrize("fmt", ["f16", "x6", "f16x8"])
def test_elbo_and_grad(device, N, M, K, D, ls, S, modified, fmt):
    """Both image formats of the chain (split-f16, the default, and split-bf16 x6),
    and split-f16 with the e4m3 cross terms in K5 and in the S_k A backward (f16x8)."""
    from modulatedgps_amd import config
    old, old_cross = config.expert_format(), config.expert_cross()
    config.set_expert_format("x6" if fmt == "x6" else "f16")
    config.set_expert_cross("f8" if fmt == "f16x8" else "f16")
    try:
        # f16x8 (e4m3 cross terms, ~9x the f32-class error of K5's term by design):
        # assign.variance's gradient is a near-cancelling sum over all N of the fvar_a
        # terms K5 produces (d fvar / d variance = 1 - ||A||^2 + ||L^T A||^2 terms of
        # opposite sign), so K5's 2^-15 per-product cross-term error shows there first:
        # 2.9-3.0e-4 normwise against float64 at config-5 shapes.  Only that block gets
        # the 4e-4 floor; every other block keeps FLOOR.
        floors = {"assign.variance": 4e-4} if fmt == "f16x8" else None
        # N = 1000, M = 25, D = 1 (inducing points on a line, cond(Kuu) ~1e7): the kernel
        # variance gradients are near-cancelling sums whose float32 error is noise at this
        # conditioning -- float32 autograd itself is 4.5e-4 off on assign.variance, and two
        # equally valid split-f16 backward variants (round 6: grad_a_c vs grad_a_c16, same
        # forward) measured 6.4e-4 and 8.7e-4 -- so this case asks for 2x, not 1.5x
        factor = 2.0 if (M, D) == (25, 1) else 1.5
        _check_elbo_and_grad(device, N, M, K, D, ls, S, modified, floors=floors, factor=factor)
    finally:
        config.set_expert_format(old)
        config.set_expert_cross(old_cross)


def test_elbo_and_grad_c3_full(device):
    """The gradient the bench's training line runs, at BASELINE config 3 in full
    (N = 65536, M = 1024, K = 8, D = 8, S = 25, lengthscale 1.0) in the default
    split-f16 format, against float64 autograd of oracle/grad_ref.py with the same
    explicit noise and the same floors as test_elbo_and_grad (the oracle takes ~1 min
    and ~25 GB on the host).  The per-block errors (HIP / float32 autograd) are printed;
    the module docstring lists them."""
    from modulatedgps_amd import config
    assert config.expert_format() == "f16" and config.expert_cross() == "f16"
    _check_elbo_and_grad(device, 65536, 1024, 8, 8, 1.0, 25, False)


def _check_elbo_and_grad(device, N, M, K, D, ls, S, modified, floor=None, floors=None, factor=1.5):
    floor = FLOOR if floor is None else floor
    floors = floors or {}
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    a_var = np.linspace(0.3, 0.9, K)[None, :] if modified else None
    z, u = R.explicit_noise(S, N, K, seed=5)
    e_ref, g_ref = _oracle(X, Y, p, z, u, a_var)
    _, g_f32 = _oracle(X, Y, p, z, u, a_var, dtype=torch.float32)
    model = _model(p, device, a_var)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e, grads = model.elbo_and_grad(Xd, Y, noise=dev_noise(z, u, device))
    assert float(e.cpu()) == pytest.approx(e_ref, rel=1e-4)
    names = [n for n, _, _ in model.trainable_parameters()]
    assert sorted(names) == sorted(g_ref)
    errs, errs32 = {}, {}
    for n in names:
        got = _dense(n, grads[n], M)
        ref = g_ref[n].reshape(got.shape)
        if np.linalg.norm(ref) < 1e-20:   # a block that is exactly (or underflows to) zero: absolute
            assert np.linalg.norm(got.astype(np.float64) - ref) < 1e-6, (n, got, ref)
            continue
        errs[n] = normwise(got, ref)
        errs32[n] = normwise(g_f32[n].reshape(got.shape), ref)
    print({k: f"{v:.1e}/{errs32[k]:.1e}" for k, v in errs.items()})
    for n, err in errs.items():
        assert err < max(floors.get(n, floor), factor * errs32[n]), (n, err, errs32[n])


def test_adam_step(device):
    """mgp_adam_step, free and softplus-positive parameters, three steps, against
    cpu_ref.adam_tf_legacy_step on the unconstrained variable (minimising -ELBO)."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(3)
    rows, cols, ld = 37, 5, 8
    lr = 0.01
    for positive in (False, True):
        theta0 = rng.uniform(0.2, 2.0, (rows, cols))
        buf = torch.zeros(rows, ld, dtype=torch.float32, device=device)
        theta = buf[:, :cols]
        theta.copy_(torch.as_tensor(theta0, dtype=torch.float32))
        th32 = theta0.astype(np.float32).astype(np.float64)
        u_ref = np.log(np.expm1(th32)) if positive else th32.copy()
        u = torch.as_tensor(u_ref, dtype=torch.float32, device=device).contiguous() if positive else None
        u_ref = u_ref.astype(np.float32).astype(np.float64)
        m1 = torch.zeros(rows, cols, dtype=torch.float32, device=device)
        m2 = torch.zeros_like(m1)
        m_ref = np.zeros((rows, cols))
        v_ref = np.zeros((rows, cols))
        for t in (1, 2, 3):
            g = rng.standard_normal((rows, cols))
            gd = torch.as_tensor(g, dtype=torch.float64 if t == 2 else torch.float32, device=device)
            ops.adam_step(theta, gd, m1, m2, t, lr, u=u)
            g32 = g.astype(np.float32).astype(np.float64)
            gu = -g32 * (1.0 / (1.0 + np.exp(-u_ref)) if positive else 1.0)
            u_ref, m_ref, v_ref = R.adam_tf_legacy_step(u_ref, gu, m_ref, v_ref, t, lr)
        th_ref = np.log1p(np.exp(u_ref)) if positive else u_ref
        assert np.abs(to_np(theta) - th_ref).max() < 1e-5 * max(1.0, np.abs(th_ref).max())
        assert np.all(to_np(buf[:, cols:]) == 0)


def test_adam_step_set_bit_identical(device):
    """mgp_adam_step_set (one launch over every block) equals one mgp_adam_step per
    block bit for bit: free and positive blocks, float and double gradients, padded
    rows, an empty block and a 1 x 1 block, three steps."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(5)
    shapes = [(37, 5, 8, False, False), (1, 1, 1, True, True), (0, 3, 4, False, False), (1024, 8, 8, False, False),
              (3, 1024, 1028, True, False), (2, 7, 7, True, True), (513, 257, 260, False, False)]

    def make():
        r = np.random.default_rng(9)
        blocks = []
        for rows, cols, ld, pos, _ in shapes:
            buf = torch.zeros(rows, ld, dtype=torch.float32, device=device)
            th = buf[:, :cols]
            th.copy_(torch.as_tensor(r.uniform(0.2, 2.0, (rows, cols)), dtype=torch.float32))
            u = (torch.log(torch.expm1(th.double())).float().contiguous() if pos else None)
            blocks.append((th, torch.zeros(rows, cols, device=device), torch.zeros(rows, cols, device=device), u))
        return blocks

    ref, got = make(), make()
    aset = ops.AdamSet(got)
    for t in (1, 2, 3):
        grads = []
        for rows, cols, ld, pos, dbl in shapes:
            g = torch.empty(rows, cols, device=device, dtype=torch.float64 if dbl else torch.float32)
            g.copy_(torch.as_tensor(rng.standard_normal((rows, cols))))
            grads.append(g)
        for (th, m1, m2, u), g in zip(ref, grads):
            if th.numel():   # (mgp_adam_step takes no NULL pointers, an empty tensor's)
                ops.adam_step(th, g, m1, m2, t, 0.01, u=u)
        aset.step(grads, t, 0.01)
    torch.cuda.synchronize()
    for j, (a, b) in enumerate(zip(ref, got)):
        for x, y in zip(a, b):
            if x is not None:
                assert torch.equal(x, y), j


def test_run_adam_improves_elbo(device):
    """utils.training_utils.run_adam drop-in: same signature / return value; the ELBO
    rises over a short run on the c1-shaped problem (minibatches of 250)."""
    from MixtureGPs.utils import print_summary
    from utils.data import Dataset
    from utils.training_utils import run_adam
    X, Y, p = R.synthetic_problem(1000, 25, 3, 1, 0.5, state="init", S=5)
    model = build_model(p, device)
    # the demos' tf.data pipeline, on HBM-resident arrays
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    Yd = torch.as_tensor(Y, dtype=torch.float32, device=device)
    it = iter(Dataset.from_tensor_slices((Xd, Yd)).shuffle(buffer_size=1000, seed=0).batch(250).repeat())
    assert "pred.q_sqrt" in print_summary(model)
    e0 = np.mean([-float(model.training_loss(next(it)).cpu()) for _ in range(10)])
    iters, elbos = run_adam(model, 60, it, 0.01)
    assert iters == list(range(5, 61, 5))
    assert np.all(np.isfinite(elbos))
    assert np.mean(elbos[-3:]) > e0
