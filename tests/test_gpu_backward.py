"""GPU parity of the backward kernels against the float64 autograd oracle
(oracle/grad_ref.py, itself checked against cpu_ref's ELBO in test_oracle.py).

Tolerance: normwise ||g - g_ref|| / ||g_ref|| <= 1e-4 for every gradient block
(float32 kernels against float64 autograd, same explicit noise)."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from oracle import grad_ref as GR
from tests.helpers import normwise, to_np

pytestmark = pytest.mark.gpu


def _oracle_grads(X, Y, p, z, u, a_var=None):  # end-to-end (used by the parameter-gradient tests)
    pred, assign, lik = GR.params_from_oracle(p)
    keep = {}
    zt = torch.tensor(np.asarray(z, np.float32).astype(np.float64))
    ut = torch.tensor(np.asarray(u, np.float32).astype(np.float64))
    av = torch.tensor(np.asarray(a_var, np.float64).reshape(-1).astype(np.float32),
                      requires_grad=True) if a_var is not None else None
    e = GR.elbo(torch.tensor(X.astype(np.float32).astype(np.float64)),
                torch.tensor(Y.astype(np.float32).astype(np.float64)), pred, assign, lik, zt, ut,
                p.num_data, assign_lik_var=av, keep=keep)
    e.backward()
    return e, keep, pred, assign, lik, av


@pytest.mark.parametrize("N,M,K,D,ls,S,modified", [(1000, 25, 3, 1, 0.5, 25, False),
                                                    (777, 33, 5, 2, 0.8, 7, False),
                                                    (1001, 25, 1, 1, 0.5, 3, False),    # K = 1, N % 4 != 0
                                                    (3, 1, 1, 1, 0.5, 1, True),
                                                    (1000, 25, 3, 1, 0.5, 25, True),
                                                    (513, 16, 8, 3, 0.9, 4, True)])
def test_elbo_terms_backward(device, N, M, K, D, ls, S, modified):
    """K6 backward: d(data term)/d(mu_f, var_f, mu_a, var_a, lik variances) at the
    device's own conditionals, against float64 autograd of the data term at the
    same (float32) values.  The conditionals enter the Gumbel-softmax at
    temperature 0.01, so the comparison is made at identical inputs."""
    from modulatedgps_amd import ops
    from tests.helpers import build_model
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    z32, u32 = np.asarray(z, np.float32), np.asarray(u, np.float32)
    a_var = np.linspace(0.3, 0.9, K).astype(np.float32) if modified else None
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    conds = [c.clone() for c in model.conditionals(Xd)]
    Y32 = Y[:, 0].astype(np.float32)
    lv = model.likelihood.likelihood.variance.reshape(-1)
    # oracle at the same float32 inputs
    leaves = [torch.tensor(to_np(c)[:, :N].T, requires_grad=True) for c in conds]
    lik = torch.tensor(lv.cpu().numpy().astype(np.float64), requires_grad=True)
    av = torch.tensor(a_var.astype(np.float64), requires_grad=True) if modified else None
    dt = GR.data_term(*leaves, torch.tensor(Y32.astype(np.float64)), lik,
                      torch.tensor(z32.astype(np.float64)), torch.tensor(u32.astype(np.float64)),
                      assign_lik_var=av)
    (dt / N).backward()
    noise = (torch.as_tensor(z32, device=device), torch.as_tensor(u32, device=device))
    avd = torch.as_tensor(a_var, device=device) if modified else None
    G, glv, glva = ops.elbo_terms_backward(*conds, torch.as_tensor(Y32, device=device), lv, S, noise=noise,
                                           scale=1.0 / N, assign_lik_var=avd)
    for i, name in enumerate(("mu_f", "var_f", "mu_a", "var_a")):
        assert normwise(to_np(G[i])[:, :N].T, leaves[i].grad.numpy()) < 1e-4, name
    assert normwise(glv.cpu().numpy(), lik.grad.numpy()) < 1e-4
    if modified:
        assert normwise(glva.cpu().numpy(), av.grad.numpy()) < 1e-4


@pytest.mark.parametrize("N,M,K,D,ls", [(2000, 64, 3, 2, 1.0), (4097, 200, 4, 3, 1.2), (8192, 256, 8, 8, 2.0)])
def test_conditional_backward(device, N, M, K, D, ls):
    """Backward of one layer's conditional: for loss = sum(G_mu * fmean + G_v * fvar)
    with random cotangents, the gradients w.r.t. q_mu, tril(q_sqrt), A (-> Kuf =
    L^-T gA and chol(Kuu) = -tril(gKuf A^T)) and the kernel variance (through
    Knn) against float64 autograd at the same A and L^-1."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(7)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    f32 = lambda a: np.asarray(a, np.float32)
    Xt, Zt = torch.as_tensor(f32(X), device=device), torch.as_tensor(f32(L["Z"]), device=device)
    var = torch.as_tensor([L["variance"]], dtype=torch.float32, device=device)
    lst = torch.as_tensor([ls], dtype=torch.float32, device=device)
    qmu = torch.as_tensor(f32(L["q_mu"]), device=device)
    qs = ops.as_padded(torch.as_tensor(f32(L["q_sqrt"])), device=device)
    Gmu = ops.padded(K, N, device)
    Gv = ops.padded(K, N, device)
    Gmu.copy_(torch.as_tensor(rng.standard_normal((K, N)).astype(np.float32)))
    Gv.copy_(torch.as_tensor(rng.standard_normal((K, N)).astype(np.float32)))
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [lst], 1e-6)
    Kfr = ops.rbf_kuf_x6(Xt, Zt, var, lst)
    Tfr = ops.split_upper_x6(LinvT[0])
    A = ops.padded(M, N, device)
    Afr, _ = ops.trsm_stats_x6(Tfr, Kfr, qmu, M, N, A=A)
    g = ops.conditional_backward_x6(Afr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N)
    # float64 autograd at the device's own A and L^-1 (the kernels under test see
    # exactly these inputs; A's own f32 error is a forward property, tested there)
    A64 = torch.tensor(to_np(A)[:, :N], requires_grad=True)
    Linv = to_np(LinvT[0]).T
    q_mu = torch.tensor(f32(L["q_mu"]).astype(np.float64), requires_grad=True)
    q_sqrt = torch.tensor(f32(L["q_sqrt"]).astype(np.float64), requires_grad=True)
    v = torch.tensor(float(np.float32(L["variance"])), dtype=torch.float64, requires_grad=True)
    fmean = (A64.T @ q_mu).T
    LTA = torch.tril(q_sqrt).transpose(1, 2) @ A64
    fvar = v - (A64 ** 2).sum(0)[None, :] + (LTA ** 2).sum(1)
    loss = (torch.tensor(to_np(Gmu)[:, :N]) * fmean).sum() + (torch.tensor(to_np(Gv)[:, :N]) * fvar).sum()
    loss.backward()
    gKuf_ref = Linv.T @ A64.grad.numpy()                   # A = L^-1 Kuf
    gLm_ref = -np.tril(gKuf_ref @ A64.detach().numpy().T)
    assert normwise(to_np(g["g_Kuf"])[:, :N], gKuf_ref) < 1e-4
    assert normwise(to_np(g["g_Lm"]), gLm_ref) < 1e-4
    assert normwise(to_np(g["g_q_mu"]), q_mu.grad.numpy()) < 1e-4
    assert normwise(to_np(g["g_q_sqrt"]), np.tril(q_sqrt.grad.numpy())) < 1e-4
    assert float(g["g_var"].cpu()) == pytest.approx(float(v.grad), rel=1e-5)


@pytest.mark.parametrize("N,M,K,D,ls", [(2000, 64, 3, 2, 1.0), (4097, 200, 4, 3, 1.2), (3000, 300, 5, 2, 1.0),
                                        (8192, 512, 8, 8, 2.0), (1500, 96, 1, 2, 1.0)])
@pytest.mark.parametrize("pattern", ["normal", "adversarial", "tiny"])
def test_conditional_backward_c_images(device, N, M, K, D, ls, pattern):
    """The split-f16 training backward from the forward's C_k = L_k^T A images
    (grad_a_c_kernel: one pipeline over all experts, the accumulator kept in units
    of the current expert's G_v and rescaled at each expert boundary).  "adversarial"
    G_v: an all-zero expert, all-zero columns, 1e-30 entries and columns whose experts
    differ by 1e12 -- the rescale chain's clamp must neither blow up nor lose the
    large terms."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(11)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    f32 = lambda a: np.asarray(a, np.float32)
    Xt, Zt = torch.as_tensor(f32(X), device=device), torch.as_tensor(f32(L["Z"]), device=device)
    var = torch.as_tensor([L["variance"]], dtype=torch.float32, device=device)
    lst = torch.as_tensor([ls], dtype=torch.float32, device=device)
    qmu = torch.as_tensor(f32(L["q_mu"]), device=device)
    qs = ops.as_padded(torch.as_tensor(f32(L["q_sqrt"])), device=device)
    gmu = rng.standard_normal((K, N)).astype(np.float32)
    gv = rng.standard_normal((K, N)).astype(np.float32)
    if pattern == "adversarial":
        gv[min(1, K - 1)] = 0.0
        gv[:, 5:40] = 0.0
        gv[0, 40:80] = 1e-30
        gv[min(2, K - 1), 80:120] *= 1e6
        gv[0, 80:120] *= 1e-6
        gv[:, 120:130] = 1e-30
    if pattern == "tiny":   # whole columns of gA ~1e-34 (per-tile image scales 2^125 .. 2^131: past f32's 2^127)
        gv[:, 200:260] *= 1e-33
        gmu[:, 200:260] *= 1e-33
        gv[:, 300:310] = 0.0
        gmu[:, 300:310] = 0.0
    Gmu, Gv = ops.padded(K, N, device), ops.padded(K, N, device)
    Gmu.copy_(torch.as_tensor(gmu))
    Gv.copy_(torch.as_tensor(gv))
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [lst], 1e-6)
    Khr = ops.rbf_kuf_x6(Xt, Zt, var, lst, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    A = ops.padded(M, N, device)
    Ahr, sth = ops.trsm_stats_x6(Thr, Khr, qmu, M, N, A=A, f16_variance=var, in_fmt="f16", cross="f16")
    Lhr = ops.split_lower_x6(qs, fmt="f16")
    Cfr = torch.empty(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=device)
    colmax = ops.colnorm_max(qs)
    ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16", c_out=(Cfr, colmax))
    g = ops.conditional_backward_x6(Ahr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N, fmt="f16", cross="f16",
                                    c_images=(Cfr, colmax, ops.image_bound(Lhr, M, K=K)))
    g_s = ops.conditional_backward_x6(Ahr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N, fmt="f16", cross="f16")
    A64 = torch.tensor(to_np(A)[:, :N], requires_grad=True)
    Linv = to_np(LinvT[0]).T
    q_sqrt = torch.tensor(f32(L["q_sqrt"]).astype(np.float64))
    LTA = torch.tril(q_sqrt).transpose(1, 2) @ A64
    fvar = -(A64 ** 2).sum(0)[None, :] + (LTA ** 2).sum(1)
    loss = (torch.tensor(gmu.astype(np.float64)) * (A64.T @ torch.tensor(f32(L["q_mu"]).astype(np.float64))).T).sum() \
        + (torch.tensor(gv.astype(np.float64)) * fvar).sum()
    loss.backward()
    gKuf_ref = Linv.T @ A64.grad.numpy()
    got = to_np(g["g_Kuf"])[:, :N]
    assert np.isfinite(got).all()
    assert normwise(got, gKuf_ref) < 1e-4
    # column-wise too: the tiny and zero-weight columns must not pick up noise
    cols = np.linalg.norm(got - gKuf_ref, axis=0) / np.maximum(np.linalg.norm(gKuf_ref, axis=0), 1e-30)
    assert np.quantile(cols, 0.99) < 1e-3
    if pattern == "tiny":   # the tiny columns relative to themselves, the zero ones exact
        tiny = np.linalg.norm(got[:, 200:260] - gKuf_ref[:, 200:260], axis=0) / np.linalg.norm(gKuf_ref[:, 200:260], axis=0)
        assert np.quantile(tiny, 0.9) < 1e-2, np.quantile(tiny, 0.9)
        assert not got[:, 300:310].any()
    assert normwise(got, to_np(g_s["g_Kuf"])[:, :N]) < 1e-4
    assert normwise(to_np(g["g_Lm"]), to_np(g_s["g_Lm"])) < 1e-4
    # the same backward on a prep of q_sqrt (mgp_conditional_backward_prep_f16c, as the
    # training step runs it beside K3): every output bit-identical
    lb = ops.image_bound(Lhr, M, K=K)
    prep = ops.conditional_backward_prep(qs, lb)
    g_p = ops.conditional_backward_x6(Ahr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N, fmt="f16", cross="f16",
                                      c_images=(Cfr, colmax, lb), prep=prep)
    for key in g:
        if torch.is_tensor(g[key]):
            assert torch.equal(g[key], g_p[key]), key
    # ... and with max |LinvT| handed in (t_bound, as the training step takes it from K3)
    tb = torch.triu(LinvT[0][:, :M]).abs().max().reshape(1).contiguous()
    g_t = ops.conditional_backward_x6(Ahr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N, fmt="f16", cross="f16",
                                      c_images=(Cfr, colmax, lb), prep=prep, t_bound=tb)
    for key in g:
        if torch.is_tensor(g[key]):
            assert torch.equal(g[key], g_t[key]), key


@pytest.mark.parametrize("M,D,ls", [(64, 2, 0.8), (200, 3, 1.0), (1024, 8, 1.0)])
def test_chol_backward(device, M, D, ls):
    """Reverse mode of Lm = chol(Kuu) against float64 autograd."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(11)
    Z = rng.standard_normal((M, D)).astype(np.float32)
    Zt = torch.as_tensor(Z, device=device)
    var = torch.tensor([0.7], device=device)
    lst = torch.tensor([ls], dtype=torch.float32, device=device)
    L, LinvT, info = ops.kuu_potrf_trtri([Zt], [var], [lst], 1e-6, want_L=True)
    gL = ops.padded(M, M, device)
    gL.copy_(torch.as_tensor(np.tril(rng.standard_normal((M, M))).astype(np.float32)))
    g = ops.chol_backward(L[0], LinvT[0], gL)
    z64 = torch.tensor(Z.astype(np.float64))
    Kuu = (GR.rbf(z64, z64, 0.7, float(np.float32(ls))) + 1e-6 * torch.eye(M, dtype=torch.float64))
    Kuu = Kuu.detach().requires_grad_(True)
    (torch.linalg.cholesky(Kuu) * torch.tensor(to_np(gL))).sum().backward()
    ref = 0.5 * (Kuu.grad + Kuu.grad.T).numpy()
    assert normwise(to_np(g), ref) < 1e-4


@pytest.mark.parametrize("M,batch", [(64, 2), (200, 2), (1024, 2), (1024, 1), (33, 3)])
def test_chol_backward_batch_bit_identical(device, M, batch):
    """mgp_chol_backward_batch (conversions, three products with Phi folded into the
    first one's store, symmetrisation; blockIdx.z = layer) equals mgp_chol_backward
    per layer bit for bit."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(M + batch)
    Ls, LinvTs, gLs = [], [], []
    for b in range(batch):
        Z = torch.as_tensor(rng.standard_normal((M, 3)).astype(np.float32), device=device)
        L, LinvT, _ = ops.kuu_potrf_trtri([Z], [torch.tensor([0.7 + 0.1 * b], device=device)],
                                          [torch.tensor([1.1], device=device)], 1e-6, want_L=True)
        gL = ops.padded(M, M, device)
        gL.copy_(torch.as_tensor(np.tril(rng.standard_normal((M, M))).astype(np.float32)))
        Ls.append(L[0]), LinvTs.append(LinvT[0]), gLs.append(gL)
    ref = [ops.chol_backward(Ls[b], LinvTs[b], gLs[b]) for b in range(batch)]
    outs = [ops.padded(M, M, device) for _ in range(batch)]
    for o in outs:
        o.fill_(float("nan"))
    got = ops.chol_backward_batch(Ls, LinvTs, gLs, outs=outs)
    torch.cuda.synchronize()
    for b in range(batch):
        assert torch.equal(got[b], ref[b]), b


@pytest.mark.parametrize("N,M,D,ard,ldx,batch", [(65536, 1024, 8, False, 0, 2), (5000, 200, 3, True, 0, 2),
                                                  (3001, 64, 16, True, 0, 2), (2500, 80, 5, True, 8, 2),
                                                  (300, 96, 4, False, 0, 1), (100, 130, 1, False, 0, 3)])
def test_rbf_backward_batch_bit_identical(device, N, M, D, ard, ldx, batch):
    """mgp_rbf_backward_batch equals, per layer, mgp_rbf_backward on the Kuf cotangent
    (accumulating onto prior values) followed by the symmetric Kuu one, bit for bit."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(N + M + D)
    dev = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=device)
    X = rng.standard_normal((N, D))
    Xd = dev(X)
    if ldx:
        Xd = torch.full((N, ldx), 7.0, device=device)
        Xd[:, :D] = dev(X)
        Xd = Xd[:, :D]
    nls = D if ard else 1
    Zs = [dev(rng.standard_normal((M, D))) for _ in range(batch)]
    var = [dev([0.6 + 0.2 * b]) for b in range(batch)]
    ls = [dev(np.linspace(0.7, 1.3, nls) + 0.1 * b) for b in range(batch)]
    gKuf = [ops.as_padded(dev(rng.standard_normal((M, N)))) for _ in range(batch)]
    gKuu = []
    for _ in range(batch):
        g = rng.standard_normal((M, M))
        gKuu.append(ops.as_padded(dev(0.5 * (g + g.T))))
    init_Z = [dev(rng.standard_normal((M, D))) for _ in range(batch)]
    init_v = [torch.tensor([0.25 * b - 0.3], dtype=torch.float64, device=device) for b in range(batch)]
    init_l = [torch.as_tensor(rng.standard_normal(nls), dtype=torch.float64, device=device) for _ in range(batch)]
    ref = []
    for b in range(batch):
        gZ, gv, gl = init_Z[b].clone(), init_v[b].clone(), init_l[b].clone()
        ops.rbf_backward(Xd, Zs[b], var[b], ls[b], gKuf[b], accumulate=True, gZ=gZ, g_var=gv, g_ls=gl)
        ops.rbf_backward(Zs[b], Zs[b], var[b], ls[b], gKuu[b], symmetric=True, accumulate=True, gZ=gZ, g_var=gv,
                         g_ls=gl)
        ref.append((gZ, gv, gl))
    gZs, gvs, gls = [t.clone() for t in init_Z], [t.clone() for t in init_v], [t.clone() for t in init_l]
    ops.rbf_backward_batch(Xd, Zs, var, ls, gKuf, gKuu, gZs, gvs, gls, accumulate=True)
    torch.cuda.synchronize()
    for b in range(batch):
        assert torch.equal(gZs[b], ref[b][0]), b
        assert torch.equal(gvs[b], ref[b][1]), b
        assert torch.equal(gls[b], ref[b][2]), b
    # accumulate 2 (the training step): gZ / g_ls overwritten (garbage before), g_var
    # added to -- equal to the per-call path from zero gZ / g_ls
    ref2 = []
    for b in range(batch):
        gZ, gv, gl = torch.zeros_like(init_Z[b]), init_v[b].clone(), torch.zeros_like(init_l[b])
        ops.rbf_backward(Xd, Zs[b], var[b], ls[b], gKuf[b], accumulate=True, gZ=gZ, g_var=gv, g_ls=gl)
        ops.rbf_backward(Zs[b], Zs[b], var[b], ls[b], gKuu[b], symmetric=True, accumulate=True, gZ=gZ, g_var=gv,
                         g_ls=gl)
        ref2.append((gZ, gv, gl))
    gZs = [torch.full_like(t, float("nan")) for t in init_Z]
    gls = [torch.full_like(t, float("nan")) for t in init_l]
    gvs = [t.clone() for t in init_v]
    ops.rbf_backward_batch(Xd, Zs, var, ls, gKuf, gKuu, gZs, gvs, gls, accumulate=2)
    torch.cuda.synchronize()
    for b in range(batch):
        assert torch.equal(gZs[b], ref2[b][0]), b
        assert torch.equal(gvs[b], ref2[b][1]), b
        assert torch.equal(gls[b], ref2[b][2]), b


@pytest.mark.parametrize("N,M,D,ard,sym,ldx", [(3000, 64, 2, False, False, 0), (5000, 200, 3, True, False, 0),
                                                (200, 200, 3, True, True, 0), (1024, 1024, 8, False, True, 0),
                                                (4000, 96, 4, True, False, 0), (3001, 64, 16, True, False, 0),
                                                (2500, 80, 5, True, False, 8), (2500, 80, 5, False, False, 0)])
def test_rbf_backward(device, N, M, D, ard, sym, ldx):
    """Reverse mode of K(Z, X) (and of K(Z, Z) with a symmetric cotangent) w.r.t.
    Z, the variance and the lengthscales against float64 autograd; D = 4, 8, 16 with
    ldx = D and D = 5 in rows of 8 take the dwordx4 point loads, the rest the dword
    loads."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(12)
    Z = rng.standard_normal((M, D)).astype(np.float32)
    X = Z if sym else rng.standard_normal((N, D)).astype(np.float32)
    N = X.shape[0]
    lsv = (np.linspace(0.7, 1.3, D) if ard else np.array([0.9])).astype(np.float32)
    gK = rng.standard_normal((M, N)).astype(np.float32)
    if sym:
        gK = 0.5 * (gK + gK.T)
    dev = lambda a: torch.as_tensor(a, device=device)
    Xd = dev(X)
    if ldx:  # X as the first D columns of rows of ldx floats
        Xd = torch.zeros(N, ldx, device=device)
        Xd[:, :D] = dev(X)
        Xd[:, D:] = 7.0  # must not enter the result
        Xd = Xd[:, :D]
    gZ, gv, gl = ops.rbf_backward(Xd, dev(Z), dev(np.float32([0.6])), dev(lsv), ops.as_padded(dev(gK)),
                                  symmetric=sym)
    z64 = torch.tensor(Z.astype(np.float64), requires_grad=True)
    v64 = torch.tensor(float(np.float32(0.6)), dtype=torch.float64, requires_grad=True)
    l64 = torch.tensor(lsv.astype(np.float64), requires_grad=True)
    x64 = z64 if sym else torch.tensor(X.astype(np.float64))
    (GR.rbf(z64, x64, v64, l64) * torch.tensor(gK.astype(np.float64))).sum().backward()
    assert normwise(to_np(gZ), z64.grad.numpy()) < 1e-4
    assert float(gv.cpu()) == pytest.approx(float(v64.grad), rel=1e-4)
    assert normwise(gl.cpu().numpy(), l64.grad.numpy()) < 1e-4


@pytest.mark.parametrize("MI,MJ,N,B,mode,weighted", [(1024, 1024, 16384, 4, 2, True), (300, 300, 5000, 3, 1, False),
                                                     (130, 70, 777, 1, 0, True), (256, 256, 256, 2, 1, False)])
def test_gram_x6(device, MI, MJ, N, B, mode, weighted):
    """x6 gram (on-the-fly split-bf16, six plane products): against float64, errors
    at float32 level (normwise <= 2e-6 incl. the f32 rounding of the weighted operand)."""
    from modulatedgps_amd import ops
    g = torch.Generator(device="cpu").manual_seed(MI + N)
    X = torch.randn(B, MI, N, generator=g)
    Y = X[:, :MJ] + 0.3 * torch.randn(B, MJ, N, generator=g) if mode else torch.randn(B, MJ, N, generator=g)
    W = torch.rand(B, N, generator=g) if weighted else None
    def pad3(t):
        d = ops.padded(t.shape[1], t.shape[2], device, batch=t.shape[0])
        d.copy_(t.to(device))
        return d if t.shape[0] > 1 else d[0]
    Xd, Yd = pad3(X), pad3(Y)
    Wd = pad3(W[:, None, :])[..., 0, :] if weighted else None
    out = ops.gram_x6(Xd, Yd, Wd, alpha=-0.5, mode=mode, N=N)
    Yw = Y.double() * (W.double()[:, None, :] if weighted else 1.0)
    ref = -0.5 * torch.einsum("bin,bjn->bij", X.double(), Yw)
    if mode == 1:
        ref = torch.tril(ref)
    elif mode == 2:
        ref = torch.tril(ref) + torch.tril(ref, -1).transpose(1, 2)
    got = to_np(out).reshape(B, MI, -1)[:, :, :MJ]
    assert normwise(got, ref.numpy()) < 2e-6
    # split-f16 variant (mgp_gram_f16) with loose bounds (4x max |X|, the exact max |Y|, |W|):
    # 22-bit operands, the same f32 accumulation
    bx = torch.tensor([4 * float(X.abs().max())], device=device)
    by = torch.tensor([float(Y.abs().max())], device=device)
    bw = torch.tensor([float(W.abs().max())], device=device) if weighted else None
    out16 = ops.gram_x6(Xd, Yd, Wd, alpha=-0.5, mode=mode, N=N, bounds=(bx, by, bw))
    got16 = to_np(out16).reshape(B, MI, -1)[:, :, :MJ]
    assert normwise(got16, ref.numpy()) < 4e-6

@pytest.mark.parametrize("MI,MJ,N,B,mode", [(1024, 1024, 16384, 4, 2), (300, 300, 5000, 3, 2), (130, 70, 777, 2, 0),
                                            (64, 64, 31, 1, 2), (256, 256, 4096, 8, 1)])
def test_gram_f16_rows(device, MI, MJ, N, B, mode):
    """The weighted gram with X as its row image (mgp_split_rows_f16 + mgp_gram_f16_rows,
    two batch entries per workgroup) is bit-identical to mgp_gram_f16 splitting X on
    the fly (same split, same fragment order, same split-K sums), and within the
    split-f16 gram's accuracy of float64 (test_gram_x6's 4e-6)."""
    from modulatedgps_amd import ops
    g = torch.Generator(device="cpu").manual_seed(7 * MI + N)
    X = torch.randn(MI, N, generator=g)
    Y = X[:MJ] if mode else torch.randn(MJ, N, generator=g)
    W = torch.rand(B, N, generator=g) - 0.3
    Xd = ops.padded(MI, N, device).copy_(X.to(device))
    Yd = Xd[:MJ] if mode else ops.padded(MJ, N, device).copy_(Y.to(device))
    Wd = ops.padded(B, N, device).copy_(W.to(device))
    bx = torch.tensor([1.5 * float(X.abs().max())], device=device)
    by = torch.tensor([float(Y.abs().max())], device=device)
    bw = torch.tensor([float(W.abs().max())], device=device)
    ref16 = ops.gram_x6(Xd, Yd, Wd, alpha=2.0, mode=mode, N=N, bounds=(bx, by, bw))
    img = ops.split_rows_f16(Xd, bx, N=N)
    got = ops.gram_x6(Xd, Yd, Wd, alpha=2.0, mode=mode, N=N, bounds=(bx, by, bw), x_rows=img)
    assert torch.equal(got, ref16)
    ref = 2.0 * torch.einsum("in,bn,jn->bij", X.double(), W.double(), Y.double())
    if mode == 1:
        ref = torch.tril(ref)
    elif mode == 2:
        ref = torch.tril(ref) + torch.tril(ref, -1).transpose(1, 2)
    got = to_np(got).reshape(B, MI, -1)[:, :, :MJ]
    assert normwise(got, ref.numpy()) < 4e-6


@pytest.mark.parametrize("MI,MJ,N,tri", [(1024, 8, 65536, False), (300, 16, 5000, False), (77, 5, 3001, False),
                                         (40, 3, 100, False), (200, 200, 4000, True), (130, 70, 777, False)])
def test_gram_f32(device, MI, MJ, N, tri):
    """mgp_gram (X Y^T over N, float32): the narrow lane-strided path for MJ <= 16
    (g_q_mu = A G_mu^T) and the f32-MFMA tiles otherwise, against float64."""
    from modulatedgps_amd import ops
    g = torch.Generator(device="cpu").manual_seed(MI * 3 + N)
    X = torch.randn(MI, N, generator=g)
    Y = X[:MJ] if tri else torch.randn(MJ, N, generator=g)
    Xd = ops.padded(MI, N, device).copy_(X.to(device))
    Yd = ops.padded(MJ, N, device).copy_(Y.to(device))
    got = ops.gram(Xd, Yd, N=N, alpha=-0.5, tri=tri)
    ref = -0.5 * X.double() @ Y.double().T
    if tri:
        ref = torch.tril(ref)
    assert normwise(to_np(got)[:, :MJ], ref.numpy()) < 2e-6
