"""Per-kernel parity of libmgp_hip (via the C-ABI, through modulatedgps_amd.ops)
against the float64 oracle.  Tolerances (fp32 kernels vs fp64 oracle):
  Kuf/Kuu: elementwise |err| <= 2e-6 * variance
  L, L^-1, A, conditional mean/var: normwise ||a-b||/||b|| <= 1e-4
  KL, data term: relative 1e-5 / 1e-4
"""
import numpy as np
import pytest
import scipy.linalg as sla
import torch

from oracle import cpu_ref as R
from oracle import philox
from tests.helpers import normwise, to_np

pytestmark = pytest.mark.gpu


def _t(x, dev):
    return torch.as_tensor(np.asarray(x), dtype=torch.float32, device=dev)


@pytest.mark.parametrize("N,M,D,ard", [(1000, 37, 1, False), (4099, 256, 2, False), (2048, 130, 8, True),
                                       (3, 5, 16, True), (1500, 64, 3, True)])
def test_rbf_kuf_kuu(device, N, M, D, ard):
    from modulatedgps_amd import ops
    rng = np.random.default_rng(N + M)
    X = rng.standard_normal((N, D))
    Z = rng.standard_normal((M, D))
    ls = rng.uniform(0.5, 2.0, D) if ard else np.array([0.8])
    var = 0.7
    Kuf = to_np(ops.rbf_kuf(_t(X, device), _t(Z, device), _t([var], device), _t(ls, device)))
    ref = R.rbf_K(Z, X, var, ls)
    assert np.abs(Kuf - ref).max() <= 2e-6 * var
    Kuu = to_np(ops.rbf_kuu(_t(Z, device), _t([var], device), _t(ls, device), 1e-6))
    refu = R.rbf_Kuu(Z, var, ls)
    assert np.abs(Kuu - refu).max() <= 2e-6 * var
    assert np.array_equal(Kuu, Kuu.T)


@pytest.mark.parametrize("M,batch", [(1, 1), (25, 2), (64, 1), (100, 2), (256, 2), (1024, 2)])
def test_potrf_trtri(device, M, batch):
    from modulatedgps_amd import ops
    rng = np.random.default_rng(M)
    As = []
    for b in range(batch):
        Z = rng.standard_normal((M, 4))
        As.append(R.rbf_Kuu(Z, 1.0, 1.5) + 1e-3 * np.eye(M))
    A = ops.padded(M, M, device, batch=batch)
    A.copy_(torch.as_tensor(np.stack(As), dtype=torch.float32))
    L, LinvT, info = ops.potrf_trtri(A)
    assert (info.cpu() == 0).all()
    for b in range(batch):
        # fp32 forward-error bound scale: cond(L) * eps32 (cond(L) = sqrt(cond(A)))
        tol = max(1e-5, 10 * np.sqrt(np.linalg.cond(As[b])) * 1.2e-7)
        Lr = np.linalg.cholesky(As[b])
        Lg = to_np(L[b])
        assert np.array_equal(np.triu(Lg, 1), np.zeros_like(Lg))
        assert normwise(Lg, Lr) < tol
        Li = sla.solve_triangular(Lr, np.eye(M), lower=True)
        Lt = to_np(LinvT[b])
        assert np.array_equal(np.tril(Lt, -1), np.zeros_like(Lt))
        assert normwise(Lt.T, Li) < tol


def test_potrf_reports_non_spd(device):
    from modulatedgps_amd import ops
    M = 130
    A = np.eye(M)
    A[70, 70] = -1.0
    At = ops.padded(M, M, device, batch=1)
    At.copy_(torch.as_tensor(A[None], dtype=torch.float32))
    _, _, info = ops.potrf_trtri(At)
    assert int(info.cpu()[0]) == 71
    with pytest.raises(Exception):
        ops.check_info(info)


@pytest.mark.parametrize("N,M,K,D,ls", [(1000, 25, 3, 1, 0.5), (8192, 256, 4, 2, 0.15),
                                         (5000, 300, 5, 3, 0.7), (16384, 1024, 8, 8, 1.0),
                                         (777, 64, 1, 2, 1.0)])
def test_conditional(device, N, M, K, D, ls):
    """K3 (fused float64 Kuu) + K1 + K4 + K5: whitened conditional vs GPflow
    base_conditional semantics.  Tolerance 1e-4 normwise where cond(Kuu) < 1e6;
    above that the float32 rounding of L^-1 alone costs ~cond(L) eps32 and the
    bound is 5e-4 (the float32-input floor measured on the CPU)."""
    from modulatedgps_amd import ops
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    mu_ref, var_ref = R.svgp_predict_f_dedup(X, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    tol = 1e-4 if np.linalg.cond(R.rbf_Kuu(L["Z"], L["variance"], ls)) < 1e6 else 5e-4
    _, LinvT, info = ops.kuu_potrf_trtri([_t(L["Z"], device)], [_t([L["variance"]], device)],
                                         [_t([ls], device)], 1e-6)
    assert int(info.cpu()[0]) == 0
    Kuf = ops.rbf_kuf(_t(X, device), _t(L["Z"], device), _t([L["variance"]], device), _t([ls], device))
    A, stats = ops.trsm_stats(LinvT[0], Kuf, _t(L["q_mu"], device))
    qs = ops.as_padded(_t(L["q_sqrt"], device))
    fm, fv = ops.expert_conditional(A, qs, stats, _t([L["variance"]], device))
    assert normwise(to_np(fm).T, mu_ref) < tol
    assert normwise(to_np(fv).T, var_ref) < tol


def test_kuu_factorisation_matches_float64(device):
    """Fused float64 Kuu + Cholesky + inverse: L and L^-1 to float32 rounding."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(0)
    Zs = [rng.standard_normal((300, 3)), rng.standard_normal((300, 3))]
    var, ls = [0.5, 0.1], [np.array([0.7]), np.array([0.5, 1.0, 1.5])]
    L, LinvT, info = ops.kuu_potrf_trtri([_t(z, device) for z in Zs], [_t([v], device) for v in var],
                                         [_t(l, device) for l in ls], 1e-6, want_L=True)
    assert (info.cpu() == 0).all()
    for b in range(2):
        Lr = np.linalg.cholesky(R.rbf_Kuu(Zs[b].astype(np.float32), var[b], ls[b]))
        Li = sla.solve_triangular(Lr, np.eye(300), lower=True)
        assert normwise(to_np(L[b]), Lr) < 1e-6
        assert normwise(to_np(LinvT[b]).T, Li) < 1e-6


@pytest.mark.parametrize("M", [300, 1024])
def test_kuu_linvt_bound_and_bounded_split(device, M):
    """mgp_kuu_potrf_trtri_ex: K3 writes max |LinvT| into the L^-T images' trailers
    (bit-exact vs the reduction of the written LinvT), and the bounded split then
    gives the same split-f16 image as mgp_split_upper_f16's own reduction."""
    from modulatedgps_amd import _lib, ops
    rng = np.random.default_rng(3)
    Zs = [_t(rng.standard_normal((M, 4)), device) for _ in range(2)]
    var, ls = [_t([0.5], device), _t([0.1], device)], [_t([0.8], device), _t([1.3], device)]
    nbytes = _lib.load().mgp_x6_lower_bytes(M, 1)
    imgs = [torch.full((nbytes,), 7, dtype=torch.uint8, device=device) for _ in range(2)]
    _, LinvT, info = ops.kuu_potrf_trtri(Zs, var, ls, 1e-6, tfr_bound_images=imgs)
    assert (info.cpu() == 0).all()
    for b in range(2):
        bound = imgs[b][nbytes - 256:nbytes - 252].view(torch.float32).item()
        ref = float(torch.triu(LinvT[b]).abs().max())
        assert bound == ref
        ops.split_upper_x6(LinvT[b], out=imgs[b], fmt="f16", bounded=True)
        own = ops.split_upper_x6(LinvT[b], fmt="f16")
        planes = (nbytes - 256) // 3072   # fragments x (f16 hi, f16 lo, unused) KiB planes
        a = imgs[b][:planes * 3072].view(planes, 3, 1024)[:, :2]
        o = own[:planes * 3072].view(planes, 3, 1024)[:, :2]
        assert torch.equal(a, o)
        assert torch.equal(imgs[b][nbytes - 256:nbytes - 252], own[nbytes - 256:nbytes - 252])


@pytest.mark.parametrize("M,dup", [(1024, 0.0), (1024, 1e-3), (700, 1e-2)])
def test_kuu_factorisation_ill_conditioned(device, M, dup):
    """K3 on badly conditioned Kuu (inducing points with near-duplicates, cond up
    to ~1e9): L and L^-1 against float64 LAPACK, to float32 output rounding
    amplified by at most cond(L) eps64."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(M)
    Z = rng.standard_normal((M, 4))
    if dup:
        Z[1::7] = Z[0::7][:len(Z[1::7])] + dup * rng.standard_normal(Z[1::7].shape)
    Z = Z.astype(np.float32)
    L, LinvT, info = ops.kuu_potrf_trtri([_t(Z, device), _t(Z, device)], [_t([0.5], device)] * 2,
                                         [_t([1.0], device)] * 2, 1e-6, want_L=True)
    assert (info.cpu() == 0).all()
    Kuu = R.rbf_Kuu(Z.astype(np.float64), 0.5, np.array([1.0]))
    Lr = np.linalg.cholesky(Kuu)
    Li = sla.solve_triangular(Lr, np.eye(M), lower=True)
    condK = np.linalg.cond(Kuu)
    for b in range(2):
        eL, eI = normwise(to_np(L[b]), Lr), normwise(to_np(LinvT[b]).T, Li)
        print(f"cond(Kuu)={condK:.2e} L {eL:.2e} Linv {eI:.2e}")
        assert eL < 1e-6 + condK * 1e-15
        assert eI < 1e-6 + condK * 1e-15


def test_conditional_ignores_upper_triangle(device):
    """band_part(q_sqrt, -1, 0): garbage above the diagonal must not matter."""
    from modulatedgps_amd import ops
    N, M, K = 600, 40, 2
    X, Y, p = R.synthetic_problem(N, M, K, 2, 0.6, state="perturbed", S=2)
    L = p.pred
    Kuu = ops.rbf_kuu(_t(L["Z"], device), _t([0.5], device), _t([0.6], device), 1e-6)
    _, LinvT, _ = ops.potrf_trtri(Kuu.unsqueeze(0))
    Kuf = ops.rbf_kuf(_t(X, device), _t(L["Z"], device), _t([0.5], device), _t([0.6], device))
    A, st = ops.trsm_stats(LinvT[0], Kuf, _t(L["q_mu"], device))
    q1 = ops.as_padded(_t(np.tril(L["q_sqrt"]), device))
    junk = np.tril(L["q_sqrt"]) + np.triu(np.random.default_rng(0).standard_normal((K, M, M)), 1)
    q2 = ops.as_padded(_t(junk, device))
    a = ops.expert_conditional(A, q1, st, _t([0.5], device))[1]
    b = ops.expert_conditional(A, q2, st, _t([0.5], device))[1]
    assert torch.equal(a, b)


@pytest.mark.parametrize("M,K", [(25, 3), (256, 4), (1024, 8), (1, 1)])
def test_gauss_kl(device, M, K):
    from modulatedgps_amd import ops
    rng = np.random.default_rng(M)
    q_mu = 0.5 * rng.standard_normal((M, K))
    q_sqrt = 0.5 * np.eye(M) + np.tril(0.1 * rng.standard_normal((K, M, M)))
    kl = float(ops.gauss_kl_white(_t(q_mu, device), ops.as_padded(_t(q_sqrt, device))).cpu())
    ref = R.gauss_kl_white(q_mu.astype(np.float32), q_sqrt.astype(np.float32))
    assert kl == pytest.approx(ref, rel=1e-5)


def test_philox_stream_bitexact(device):
    """The device noise stream equals oracle/philox.py (uniforms bit-exact, normals ~1 ulp)."""
    from modulatedgps_amd import ops
    seed, S, N, K = 0x1234ABCD9876, 3, 1000, 7
    z, u = ops.philox_noise(seed, 500, N, K, S, device)
    uref = philox.noise_uniform(seed, S, np.arange(500, 500 + N), K)
    zref = philox.noise_normal(seed, S, np.arange(500, 500 + N), K)
    assert np.array_equal(to_np(u), uref.astype(np.float32).astype(np.float64))
    assert np.abs(to_np(z) - zref).max() < 2e-5
    z2 = ops.philox_normal2(seed, 500, N, K, S, device)
    assert np.abs(to_np(z2) - philox.noise_normal(seed, S, np.arange(500, 500 + N), K, stream=2)).max() < 2e-5


@pytest.mark.parametrize("N,K,S", [(1000, 3, 25), (4097, 8, 5), (300, 1, 4), (513, 16, 2)])
def test_elbo_terms_explicit_and_philox(device, N, K, S):
    from modulatedgps_amd import ops
    rng = np.random.default_rng(N)
    mu_f, mu_a = rng.standard_normal((2, N, K))
    var_f, var_a = rng.uniform(0.05, 1.0, (2, N, K))
    Y = rng.standard_normal((N, 1))
    lv = rng.uniform(0.2, 1.0, (1, K))
    z, u = R.explicit_noise(S, N, K, seed=3)

    def ref(z, u):
        W = R.assignment_weights(mu_a[None], var_a[None], z, u)
        return np.sum(R.e_log_p_y(mu_f[None], var_f[None], Y, lv, W, S))

    dev = lambda a: ops.as_padded(_t(a.T, device))
    args = (dev(mu_f), dev(var_f), dev(mu_a), dev(var_a), _t(Y[:, 0], device), _t(lv[0], device), S)
    out = float(ops.elbo_terms(*args, noise=(_t(z, device), _t(u, device))).cpu())
    r = ref(z, u)
    assert out == pytest.approx(r, rel=1e-4, abs=1e-3)
    seed = 99
    out2 = float(ops.elbo_terms(*args, seed=seed).cpu())
    n = np.arange(N)
    r2 = ref(philox.noise_normal(seed, S, n, K), philox.noise_uniform(seed, S, n, K))
    assert out2 == pytest.approx(r2, rel=1e-4, abs=1e-3)


def test_elbo_terms_rounding_negative_assign_var(device):
    """A float32 marginal variance of the assign layer can round below -jitter
    where the reference's float64 one sits at ~0 (seen in demo_tf2_modified_
    multiclass after ~1400 Adam steps: the sqrt of the reparameterisation went
    NaN and so did the step).  K6 samples with sqrt(max(var + jitter, 0)): equal
    to the oracle on the clamped variances, the reference's own value on
    (-jitter, 0], and the backward stays finite with a zero variance gradient
    only where the clamp is active."""
    from modulatedgps_amd import ops
    N, K, S = 1000, 3, 25
    rng = np.random.default_rng(5)
    mu_f, mu_a = rng.standard_normal((2, N, K))
    var_f, var_a = rng.uniform(0.05, 1.0, (2, N, K))
    var_a[::7, 1] = -3e-6                      # below -jitter (1e-6)
    var_a[3::7, 2] = -5e-7                     # inside (-jitter, 0]: the reference is finite there
    Y = rng.standard_normal((N, 1))
    lv = rng.uniform(0.2, 1.0, (1, K))
    z, u = R.explicit_noise(S, N, K, seed=3)
    W = R.assignment_weights(mu_a[None], np.maximum(var_a, -R.JITTER)[None], z, u)
    r = np.sum(R.e_log_p_y(mu_f[None], var_f[None], Y, lv, W, S))
    dev = lambda a: ops.as_padded(_t(a.T, device))
    args = (dev(mu_f), dev(var_f), dev(mu_a), dev(var_a), _t(Y[:, 0], device), _t(lv[0], device), S)
    noise = (_t(z, device), _t(u, device))
    out = float(ops.elbo_terms(*args, noise=noise).cpu())
    assert np.isfinite(out) and out == pytest.approx(r, rel=1e-4, abs=1e-3)
    G = ops.elbo_terms_backward(*args, noise=noise)[0].float().cpu().numpy()
    assert np.all(np.isfinite(G[:, :K, :N]))
    assert np.all(G[3, 1, :N:7] == 0.0)
    assert np.count_nonzero(G[3, 2, 3:N:7]) > 0.9 * len(range(3, N, 7))


@pytest.mark.parametrize("N,M,K,D,ls", [(1000, 25, 3, 1, 0.5), (8192, 256, 4, 2, 0.15),
                                         (5000, 300, 5, 3, 0.7), (16384, 1024, 8, 8, 1.0),
                                         (777, 64, 1, 2, 1.0)])
def test_conditional_split_bf16(device, N, M, K, D, ls):
    """K5 on split-bf16 fragment images (x6): same bound as the f32 path against
    the float64 oracle, and within 2e-6 normwise of the exact-f32 MFMA K5."""
    from modulatedgps_amd import ops
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    mu_ref, var_ref = R.svgp_predict_f_dedup(X, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    tol = 1e-4 if np.linalg.cond(R.rbf_Kuu(L["Z"], L["variance"], ls)) < 1e6 else 5e-4
    _, LinvT, info = ops.kuu_potrf_trtri([_t(L["Z"], device)], [_t([L["variance"]], device)],
                                         [_t([ls], device)], 1e-6)
    Kuf = ops.rbf_kuf(_t(X, device), _t(L["Z"], device), _t([L["variance"]], device), _t([ls], device))
    A, stats = ops.trsm_stats(LinvT[0], Kuf, _t(L["q_mu"], device))
    qs = ops.as_padded(_t(L["q_sqrt"], device))
    var = _t([L["variance"]], device)
    fm32, fv32 = ops.expert_conditional(A, qs, stats, var)
    Afr = ops.split_cols_x6(A)
    Lfr = ops.split_lower_x6(qs)
    fm, fv = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K)
    assert torch.equal(fm[:, :N], fm32[:, :N])
    assert normwise(to_np(fv).T, to_np(fv32).T) < 2e-6
    assert normwise(to_np(fm).T, mu_ref) < tol
    assert normwise(to_np(fv).T, var_ref) < tol


def test_split_bf16_layout_exact(device):
    """Operands exactly representable in bf16 (small integers): the split is
    exact (mid = lo = 0), so the x6 sum of squares must match float64 to f32
    rounding of the final sums -- catches any k-order / lane-map mismatch."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(3)
    M, N, K = 256, 512, 2
    A = rng.integers(-3, 4, size=(M, N)).astype(np.float32)
    Ls = np.tril(rng.integers(-2, 3, size=(K, M, M))).astype(np.float32)
    At, qs = _t(A, device), ops.as_padded(_t(Ls, device))
    stats = torch.zeros(ops.stats_tiles(M), K + 1, N, device=device)
    fm, fv = ops.expert_conditional_x6(ops.split_cols_x6(At), ops.split_lower_x6(qs), stats,
                                       _t([0.0], device), M, N, K)
    ref = np.stack([np.sum((Ls[k].T.astype(np.float64) @ A) ** 2, axis=0) for k in range(K)])
    assert np.array_equal(to_np(fv)[:, :N].astype(np.float64), ref)


@pytest.mark.parametrize("N,M,D,K", [(8192, 256, 2, 4), (1000, 25, 1, 3), (777, 300, 3, 16),
                                     (4096, 1024, 8, 8)])
def test_kuf_and_trsm_images(device, N, M, D, K):
    """K1 -> Kuf image and K4 on images (x6).  Kuf: the decoded image is within
    the f32 rounding bound of GPflow's expanded square-distance formula.  A = L^-1 Kuf and the
    stats: against float64 (oracle Kuu, LAPACK), the x6 error is no larger than
    the exact-f32 MFMA K4's (A is ill-conditioned: cond(L) amplifies any
    rounding, so "equal to the f32 kernel" is not a meaningful bound).  The
    padding of the A image is zero."""
    from modulatedgps_amd import ops
    from tests.helpers import decode_cols_image
    X, Y, p = R.synthetic_problem(N, M, K, D, 0.7, state="perturbed", S=2)
    L = p.pred
    Xt, Zt, var, ls = _t(X, device), _t(L["Z"], device), _t([L["variance"]], device), _t([0.7], device)
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [ls], 1e-6)
    Kuf = ops.rbf_kuf(Xt, Zt, var, ls)
    A, st = ops.trsm_stats(LinvT[0], Kuf, _t(L["q_mu"], device))
    Kfr = torch.full((ops.x6_cols_bytes(M, N),), 0x7F, dtype=torch.uint8, device=device)
    Kfr = ops.rbf_kuf_x6(Xt, Zt, var, ls, out=Kfr)
    kd = decode_cols_image(Kfr, M, N)
    z64, x64 = L["Z"].astype(np.float32).astype(np.float64), X.astype(np.float32).astype(np.float64)
    k64 = R.rbf_K(z64, x64, L["variance"], 0.7)
    # the image kernel evaluates GPflow's expanded form |z'|^2 + |x'|^2 - 2 z'.x'
    # (z' = z sqrt(0.5 log2 e) / l) with the cross term on the f32 MFMA: its f32
    # rounding error is a few eps32 (|z'|^2 + |x'|^2) in the exponent
    c2 = 0.5 * np.log2(np.e) / 0.7 ** 2
    norms = c2 * (np.sum(z64 ** 2, 1)[:, None] + np.sum(x64 ** 2, 1)[None, :])
    bound = 2e-6 * L["variance"] + k64 * np.log(2.0) * 8 * 2.0 ** -24 * norms
    assert np.all(np.abs(kd - k64) <= bound)
    Tfr = ops.split_upper_x6(LinvT[0])
    Afr, st6 = ops.trsm_stats_x6(Tfr, Kfr, _t(L["q_mu"], device), M, N)
    L64 = np.linalg.cholesky(R.rbf_Kuu(L["Z"].astype(np.float32).astype(np.float64), L["variance"], 0.7))
    A64 = sla.solve_triangular(L64, R.rbf_K(L["Z"].astype(np.float32).astype(np.float64),
                                            X.astype(np.float32).astype(np.float64), L["variance"], 0.7),
                               lower=True)
    e32 = normwise(to_np(A), A64)
    e6 = normwise(decode_cols_image(Afr, M, N), A64)
    assert e6 <= max(1.5 * e32, 2e-6), (e6, e32)
    T = st.shape[0]
    q64 = L["q_mu"].astype(np.float32).astype(np.float64)
    ref = np.zeros((T, K + 1, N))
    for t in range(T):
        rows = slice(64 * t, min(64 * t + 64, M))
        ref[t, 0] = np.sum(A64[rows] ** 2, axis=0)
        ref[t, 1:] = q64[rows].T @ A64[rows]
    s32 = normwise(to_np(st)[:, :, :N], ref)
    s6 = normwise(to_np(st6)[:, :, :N], ref)
    assert s6 <= max(1.5 * s32, 2e-6), (s6, s32)
    Mp, Np = -(-M // 128) * 128, -(-N // 256) * 256
    full = decode_cols_image(Afr, Mp, Np)
    assert not full[M:].any() and not full[:, N:].any()


def test_expert_conditional_planes(device):
    """K5 on 3 / 2 / 1 bf16 planes (mgp_expert_conditional_planes): 3 planes are
    bit-identical to the x6 entry; the reduced modes (BASELINE config 5's "bf16
    mixed") are measured against the float64 oracle: 2 planes within the 1e-4
    gate, 1 plane (bf16 operands) within 1e-2."""
    from modulatedgps_amd import ops
    N, M, K, D, ls = 8192, 1024, 8, 8, 1.0
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    mu_ref, var_ref = R.svgp_predict_f_dedup(X, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    var = _t([L["variance"]], device)
    lsc = _t([ls], device)
    Zt = _t(L["Z"], device)
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [lsc], 1e-6)
    Kfr = ops.rbf_kuf_x6(_t(X, device), Zt, var, lsc)
    Tfr = ops.split_upper_x6(LinvT[0])
    Afr, stats = ops.trsm_stats_x6(Tfr, Kfr, _t(L["q_mu"], device), M, N)
    Lfr = ops.split_lower_x6(ops.as_padded(_t(L["q_sqrt"], device)))
    fm6, fv6 = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K)
    fm6, fv6 = to_np(fm6), to_np(fv6)
    errs = {}
    for planes, tol in ((3, 1e-4), (2, 1e-4), (1, 1e-2)):
        fm, fv = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K, planes=planes)
        fm, fv = to_np(fm), to_np(fv)
        if planes == 3:
            assert np.array_equal(fv, fv6) and np.array_equal(fm, fm6)
        errs[planes] = normwise(fv.T, var_ref)
        assert normwise(fm.T, mu_ref) < 1e-4  # fmean comes from K4 (x6) in every mode
        assert errs[planes] < tol, (planes, errs[planes])
    print("K5 planes fvar normwise error vs float64:", errs)


@pytest.mark.parametrize("N,M,D,ard", [(65536, 1024, 8, False), (4099, 130, 3, True), (777, 300, 1, False),
                                       (1000, 40, 2, False), (513, 256, 20, True)])
@pytest.mark.parametrize("fmt", ["f16", "x6"])
def test_kuu_potrf_trtri_kuf_side_job(device, N, M, D, ard, fmt):
    """mgp_kuu_potrf_trtri_kuf: the Kuf images K(Z_b, X) of both layers written by extra
    workgroups of K3's step launches (M = 40: no step launches, K1's own launches) are
    byte-identical to mgp_rbf_kuf_f16 / mgp_rbf_kuf_x6's (trailer included), and L, L^-T
    and info are those of the factorisation without the job.  c3's shape in full first."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(N + M + D)
    X = _t(rng.standard_normal((N, D)), device)
    Zs = [_t(rng.standard_normal((M, D)), device) for _ in range(2)]
    var = [_t([0.7], device), _t([0.3], device)]
    ls = [_t(rng.uniform(0.8, 2.0, D) if ard else [1.1], device), _t(rng.uniform(0.8, 2.0, D) if ard else [0.9], device)]
    nbytes = ops._lib.load().mgp_x6_cols_bytes(M, N)
    ref = [torch.zeros(nbytes, dtype=torch.uint8, device=device) for _ in range(2)]
    got = [torch.zeros(nbytes, dtype=torch.uint8, device=device) for _ in range(2)]
    for b in range(2):
        ops.rbf_kuf_x6(X, Zs[b], var[b], ls[b], out=ref[b], fmt=fmt)
    L0, LinvT0, info0 = ops.kuu_potrf_trtri(Zs, var, ls, 1e-6, want_L=True)
    L1, LinvT1, info1 = ops.kuu_potrf_trtri(Zs, var, ls, 1e-6, want_L=True, kuf=(X, got, fmt))
    torch.cuda.synchronize()
    for b in range(2):
        assert torch.equal(got[b], ref[b]), b
    assert torch.equal(L1, L0) and torch.equal(LinvT1, LinvT0) and torch.equal(info1, info0)


@pytest.mark.parametrize("M,K,batch", [(1024, 8, 2), (130, 5, 2), (40, 2, 2), (300, 3, 1), (1, 1, 2)])
def test_qsqrt_images_kl_batch_bit_identical(device, M, K, batch):
    """mgp_qsqrt_images_kl_f16_batch: both layers' split-f16 tril(q_sqrt) images (fragments and
    the trailer's bound) byte-identical to mgp_split_lower_f16's, KL terms equal to
    mgp_gauss_kl_white's; q_sqrt carries garbage above the diagonal."""
    from modulatedgps_amd import ops
    rng = np.random.default_rng(M + 11 * K)
    q_mu = [_t(0.5 * rng.standard_normal((M, K)), device) for _ in range(batch)]
    q_sqrt = []
    for b in range(batch):
        q = ops.padded(M, M, device, batch=K)
        q.copy_(_t(np.eye(M) * (0.5 + b) + 0.1 * rng.standard_normal((K, M, M)), device))
        q_sqrt.append(q)
    lb = ops.x6_lower_bytes(M, K)
    ref = [ops.split_lower_x6(q_sqrt[b], fmt="f16") for b in range(batch)]
    kl_ref = [ops.gauss_kl_white(q_mu[b], q_sqrt[b]) for b in range(batch)]
    got = [torch.full((lb,), 7, dtype=torch.uint8, device=device) for _ in range(batch)]
    kl = [torch.full((1,), float("nan"), dtype=torch.float64, device=device) for _ in range(batch)]
    ops.qsqrt_images_kl_f16_batch(q_mu, q_sqrt, got, kl)
    torch.cuda.synchronize()
    Mp = (M + 127) // 128 * 128
    nfb = K * (Mp // 32) * (Mp // 16) * 3 * 1024   # the fragments' bytes (the trailer's bound after them)
    for b in range(batch):
        assert torch.equal(got[b][:nfb], ref[b][:nfb]), b
        assert torch.equal(got[b][lb - 256:lb - 252], ref[b][lb - 256:lb - 252]), b
        assert torch.equal(kl[b], kl_ref[b]), (b, kl[b].item(), kl_ref[b].item())
