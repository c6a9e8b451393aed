"""Split-f16 ("f16x3") forward chain (mgp_rbf_kuf_f16, mgp_split_upper_f16,
mgp_trsm_stats_f16 / mgp_trsm_stats_x6_f16, mgp_split_lower_f16 /
mgp_split_cols_f16, mgp_expert_conditional_f16) against
the float64 oracle, at the north_star gate (ELBO 1e-4 relative, fmean/fvar 1e-4
normwise) and against the split-bf16 x6 path's own error."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from tests.helpers import build_model, decode_cols_f16, dev_noise, load_golden, normwise, params_from_golden, to_np

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["x6", "f16", "f16x8"])
def fmt_mode(request):
    """Both forward image formats end to end, and the split-f16 K5 with its cross
    terms on the e4m3 MFMA (tests/test_gpu_model.py runs the default one)."""
    from modulatedgps_amd import config
    old, old_cross = config.expert_format(), config.expert_cross()
    config.set_expert_format("x6" if request.param == "x6" else "f16")
    config.set_expert_cross("f8" if request.param == "f16x8" else "f16")
    yield request.param
    config.set_expert_format(old)
    config.set_expert_cross(old_cross)


def _t(a, device):
    return torch.as_tensor(np.asarray(a, np.float32), device=device)


def _k5_only(ops, A, qs, M, N, K, fmt, device, cross="f16"):
    """K5's own term: fvar = sum_m' (L^T A)^2 with zero stats and zero variance."""
    Afr = ops.split_cols_x6(A, fmt=fmt)
    Lfr = ops.split_lower_x6(qs, fmt=fmt)
    T = ops.stats_tiles(M)
    stats = ops.padded(T * (K + 1), N, device).unflatten(0, (T, K + 1))
    stats.zero_()
    zero = torch.zeros(1, dtype=torch.float32, device=device)
    fm, fv = ops.expert_conditional_x6(Afr, Lfr, stats, zero, M, N, K, fmt=fmt, cross=cross)
    return to_np(fm), to_np(fv)


@pytest.mark.parametrize("sa,sl", [(1.0, 1.0), (3e-4, 7e2), (2.0 ** 20, 2.0 ** -18), (1e3, 1e-5)])
def test_expert_f16_scale_invariance(device, sa, sl):
    """Ragged M, N; operands far from unit scale: the power-of-two image scale
    keeps the split-f16 K5 at its relative accuracy whatever the magnitudes."""
    from modulatedgps_amd import ops
    M, N, K = 200, 1000, 3
    rng = np.random.default_rng(3)
    A = rng.standard_normal((M, N)) * sa
    qs = np.tril(rng.standard_normal((K, M, M))) * sl
    qs += np.triu(np.full((M, M), 1e30), 1)          # upper triangle is ignored (band_part)
    A32, qs32 = A.astype(np.float32), qs.astype(np.float32)
    ref = np.einsum("kmi,mn->kin", np.tril(qs32.astype(np.float64)), A32.astype(np.float64))
    ref = (ref ** 2).sum(1)                         # [K, N]
    Ad = ops.as_padded(_t(A32, device))
    qd = ops.as_padded(_t(qs32, device))
    fm, fv = _k5_only(ops, Ad, qd, M, N, K, "f16", device)
    assert np.all(fm == 0)
    err16 = normwise(fv, ref)
    _, fv6 = _k5_only(ops, Ad, qd, M, N, K, "x6", device)
    err6 = normwise(fv6, ref)
    fm8, fv8 = _k5_only(ops, Ad, qd, M, N, K, "f16", device, cross="f8")
    err8 = normwise(fv8, ref)
    print(f"scale ({sa:g}, {sl:g}): f16x3 {err16:.2e}  f16x8 {err8:.2e}  x6 {err6:.2e}")
    assert err16 < 3e-7 and err16 < 1.5 * err6       # measured 1.0e-7 (x6 1.0e-7) at every scale
    assert np.all(np.isfinite(fv)) and np.all(np.isfinite(fv8)) and np.all(fm8 == 0)
    assert err8 < 1e-5


def test_expert_conditional_f16_accuracy(device):
    """Config-3 shapes at reduced N: K4 (x6 inputs, split-f16 A image) -> K5 f16
    against the float64 oracle, beside the x6 path."""
    from modulatedgps_amd import ops
    N, M, K, D, ls = 8192, 1024, 8, 8, 1.0
    X, _, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    mu_ref, var_ref = R.svgp_predict_f_dedup(X, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    var, lsc, Zt = _t([L["variance"]], device), _t([ls], device), _t(L["Z"], device)
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [lsc], 1e-6)
    Kfr = ops.rbf_kuf_x6(_t(X, device), Zt, var, lsc)
    Tfr = ops.split_upper_x6(LinvT[0])
    qm, qs = _t(L["q_mu"], device), ops.as_padded(_t(L["q_sqrt"], device))
    errs = {}
    for fmt in ("x6", "f16"):
        Afr, stats = ops.trsm_stats_x6(Tfr, Kfr, qm, M, N, f16_variance=var if fmt == "f16" else None)
        Lfr = ops.split_lower_x6(qs, fmt=fmt)
        fm, fv = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K, fmt=fmt)
        errs[fmt] = (normwise(to_np(fm).T, mu_ref), normwise(to_np(fv).T, var_ref))
    # the whole forward chain in split-f16: K1 (mgp_rbf_kuf_f16), L^-T image
    # (mgp_split_upper_f16), K4 on f16 inputs (mgp_trsm_stats_f16), K5 f16
    Khr = ops.rbf_kuf_x6(_t(X, device), Zt, var, lsc, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    Afr, stats = ops.trsm_stats_x6(Thr, Khr, qm, M, N, f16_variance=var, in_fmt="f16")
    fm, fv = ops.expert_conditional_x6(Afr, ops.split_lower_x6(qs, fmt="f16"), stats, var, M, N, K, fmt="f16")
    errs["f16 chain"] = (normwise(to_np(fm).T, mu_ref), normwise(to_np(fv).T, var_ref))
    Afr, stats = ops.trsm_stats_x6(Thr, Khr, qm, M, N, f16_variance=var, in_fmt="f16", cross="f8")
    fm, fv = ops.expert_conditional_x6(Afr, ops.split_lower_x6(qs, fmt="f16"), stats, var, M, N, K, fmt="f16",
                                       cross="f8")
    errs["f16x8 chain"] = (normwise(to_np(fm).T, mu_ref), normwise(to_np(fv).T, var_ref))
    print("fmean / fvar normwise error vs float64:", errs)
    # fmean comes from K4's stats: float32 VALU sums (x6) vs split-f16 MFMAs (f16),
    # both float32-class (measured 1.016e-6 vs 1.011e-6)
    assert errs["f16"][0] < 1.05 * errs["x6"][0]
    assert errs["f16"][1] < 1e-4
    assert errs["f16"][1] < 1.5 * errs["x6"][1]        # measured 7.34e-7 vs x6 7.31e-7
    assert errs["f16 chain"][0] < 1e-4 and errs["f16 chain"][1] < 1e-4
    assert errs["f16 chain"][0] < 8 * errs["x6"][0] and errs["f16 chain"][1] < 8 * errs["x6"][1]
    # fmean from K4's stats: the f16x8 chain's K4 is the 32x32x16 kernel, the f16 chain's
    # the 16x16x32 one (trsm_stats16_kernel) -- the same products in another summation order
    assert errs["f16x8 chain"][0] == pytest.approx(errs["f16 chain"][0], rel=0.05)
    assert errs["f16x8 chain"][1] < 1e-4


@pytest.mark.parametrize("case", ["case_demo_init", "case_demo_perturbed", "case_c1"])
def test_golden_elbo_formats(device, fmt_mode, case):
    d = load_golden(case + ".npz")
    p = params_from_golden(d)
    model = build_model(p, device)
    X = torch.as_tensor(d["X"], dtype=torch.float32, device=device)
    Y = torch.as_tensor(d["Y"], dtype=torch.float32, device=device)
    elbo = float(model._build_likelihood(X, Y, noise=dev_noise(d["z"], d["u"], device)).cpu())
    assert elbo == pytest.approx(float(d["elbo"]), rel=1e-4)
    mu_f, var_f, mu_a, var_a = model.conditionals(X)
    assert normwise(to_np(var_f).T, d["var_f"]) < 1e-4
    assert normwise(to_np(var_a).T, d["var_a"]) < 1e-4
    Xt = torch.as_tensor(d["Xtest"], dtype=torch.float32, device=device)
    ym, yv = model.predict_y(Xt)
    assert normwise(to_np(yv), d["predict_y_var"]) < 1e-4


@pytest.mark.parametrize("N,M,K,D,ls,S", [(8192, 256, 4, 2, 0.15, 25),      # BASELINE config 2
                                           (8192, 1024, 8, 8, 1.0, 25),      # config-3 shapes, N reduced
                                           (4096, 2048, 16, 16, 2.0, 25),    # config-5 shapes, N reduced
                                           (1001, 33, 2, 3, 0.8, 7)])        # ragged sizes
def test_elbo_configs_formats(device, fmt_mode, N, M, K, D, ls, S):
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    ref, parts = R.smgp_elbo(X, Y, p, z, u, return_parts=True)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    assert e == pytest.approx(ref, rel=1e-4)
    mu_f, var_f, mu_a, var_a = model.conditionals(Xd)
    assert normwise(to_np(mu_f).T, parts["mu_f"]) < 1e-4
    assert normwise(to_np(var_f).T, parts["var_f"]) < 1e-4
    assert normwise(to_np(mu_a).T, parts["mu_a"]) < 1e-4
    assert normwise(to_np(var_a).T, parts["var_a"]) < 1e-4


def test_mfma_shape_switches(device):
    """The split-f16 K4 and K5 on 16x16x32 MFMAs (trsm_stats16_kernel,
    expert_cond16_kernel: the only split-f16 f16x3 kernels since round 4, when the
    32x32x16 environment switches were removed from the library) against the float64
    oracle at config-3 shapes (ragged N): the forward and the training K5 that also
    writes the C_k images."""
    from modulatedgps_amd import ops
    N, M, K, D, ls = 3001, 1024, 8, 8, 1.0
    X, _, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    mu_ref, var_ref = R.svgp_predict_f_dedup(X, L["Z"], L["variance"], L["lengthscales"], L["q_mu"], L["q_sqrt"])
    var, lsc, Zt = _t([L["variance"]], device), _t([ls], device), _t(L["Z"], device)
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [lsc], 1e-6)
    qm, qs = _t(L["q_mu"], device), ops.as_padded(_t(L["q_sqrt"], device))
    Khr = ops.rbf_kuf_x6(_t(X, device), Zt, var, lsc, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    A32 = ops.padded(M, N, device)
    Afr, stats = ops.trsm_stats_x6(Thr, Khr, qm, M, N, A=A32, f16_variance=var, in_fmt="f16", cross="f16")
    Lfr = ops.split_lower_x6(qs, fmt="f16")
    fm, fv = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K, fmt="f16", cross="f16")
    assert normwise(to_np(fm).T, mu_ref) < 1e-4 and normwise(to_np(fv).T, var_ref) < 1e-4
    Cfr = torch.empty(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=device)
    fmc, fvc = ops.expert_conditional_x6(Afr, Lfr, stats, var, M, N, K, fmt="f16", cross="f16",
                                         c_out=(Cfr, ops.colnorm_max(qs)))
    assert normwise(to_np(fvc).T, var_ref) < 1e-4
    assert normwise(to_np(fvc), to_np(fv)) < 1e-6


@pytest.mark.parametrize("N,M,K,with_a", [(65536, 1024, 8, False), (8192, 256, 4, True), (3000, 200, 3, True),
                                           (8192, 1024, 8, False)])   # c4's per-rank shape: unpaired items
def test_trsm_stats_f16_batch_bit_identical(device, N, M, K, with_a):
    """mgp_trsm_stats_f16_batch (both layers' K4 in one launch) writes the same A
    images, statistics and f32 A bits as one mgp_trsm_stats_f16 call per layer,
    including ragged M and N (models.py:141-143 for pred_layer and assign_layer)."""
    from modulatedgps_amd import ops
    g = torch.Generator(device=device).manual_seed(11)
    D = 4
    X = torch.randn(N, D, device=device, generator=g)
    per = []
    for b in range(2):
        Z = torch.randn(M, D, device=device, generator=g)
        var = torch.tensor([0.7 + 0.2 * b], device=device)
        ls = torch.tensor([1.0 + 0.5 * b], device=device)
        _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
        q_mu = torch.randn(M, K, device=device, generator=g)
        Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
        Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
        per.append((Thr, Khr, q_mu, var))
    ref = []
    for Thr, Khr, q_mu, var in per:
        A = ops.padded(M, N, device) if with_a else None
        Afr, st = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, A=A, f16_variance=var, in_fmt="f16", cross="f16")
        ref.append((Afr.clone(), st.clone(), None if A is None else A.clone()))
    Afrs = [torch.full_like(r[0], 0x7F) for r in ref]
    sts = [torch.full_like(r[1], float("nan")) for r in ref]
    As = [torch.full_like(r[2], float("nan")) for r in ref] if with_a else None
    out = ops.trsm_stats_f16_batch([p[0] for p in per], [p[1] for p in per], [p[2] for p in per], M, N, Afrs, sts,
                                   [p[3] for p in per], As=As)
    torch.cuda.synchronize()
    # fragment planes 0-1 (f16 hi, lo; plane 2 is the f16x8 K4's) and the trailer's scale bound
    planes = ops.x6_cols_bytes(M, N) - 256
    for b in range(2):
        got, exp = out[b][0], ref[b][0]
        assert torch.equal(got[:planes].view(-1, 3, 64 * 16)[:, :2], exp[:planes].view(-1, 3, 64 * 16)[:, :2])
        assert torch.equal(got[planes:planes + 4], exp[planes:planes + 4])
        assert torch.equal(out[b][1][..., :N], ref[b][1][..., :N])
        if with_a:
            assert torch.equal(As[b][:, :N], ref[b][2][:, :N])


@pytest.mark.parametrize("N,M,K,train", [(65536, 1024, 8, False), (8192, 256, 4, True), (3000, 200, 3, True),
                                         (2800, 200, 3, False), (2800, 130, 2, True)])   # odd column-tile counts
def test_expert_conditional_f16_batch_bit_identical(device, N, M, K, train):
    """mgp_expert_conditional_f16_batch (both layers' K5 in one launch, forward or with
    the training C_k images) gives the same fmean / fvar / C_k bits as one
    mgp_expert_conditional_f16(c) call per layer (models.py:141-143, both layers)."""
    from modulatedgps_amd import ops
    g = torch.Generator(device=device).manual_seed(5)
    D = 4
    X = torch.randn(N, D, device=device, generator=g)
    per = []
    for b in range(2):
        Z = torch.randn(M, D, device=device, generator=g)
        var = torch.tensor([0.6 + 0.3 * b], device=device)
        ls = torch.tensor([0.9 + 0.4 * b], device=device)
        _, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
        q_mu = torch.randn(M, K, device=device, generator=g)
        qs = ops.padded(M, M, device, batch=K)
        qs.copy_(0.4 * torch.eye(M, device=device) + torch.tril(0.05 * torch.randn(K, M, M, device=device,
                                                                                     generator=g)))
        Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
        Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
        Afr, st = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, f16_variance=var, in_fmt="f16", cross="f16")
        Lhr = ops.split_lower_x6(qs, fmt="f16")
        c_out = None
        if train:
            c_out = (torch.zeros(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=device), ops.colnorm_max(qs))
        per.append((Afr, Lhr, st, var, c_out))
    ref = []
    for Afr, Lhr, st, var, c_out in per:
        fm, fv = ops.expert_conditional_x6(Afr, Lhr, st, var, M, N, K, fmt="f16", cross="f16", c_out=c_out)
        ref.append((fm.clone(), fv.clone(), None if c_out is None else c_out[0].clone()))
    fms = [ops.padded(K, N, device) for _ in range(2)]
    fvs = [ops.padded(K, N, device) for _ in range(2)]
    for t in fms + fvs:
        t.fill_(float("nan"))
    wss = [torch.empty(ops.expert_x6_workspace_bytes(M, N, K), dtype=torch.uint8, device=device) for _ in range(2)]
    c_outs = None
    if train:
        c_outs = [(torch.zeros_like(p[4][0]), p[4][1]) for p in per]
    ops.expert_conditional_f16_batch([p[0] for p in per], [p[1] for p in per], [p[2] for p in per],
                                     [p[3] for p in per], M, N, K, fms, fvs, wss, c_outs=c_outs)
    torch.cuda.synchronize()
    for b in range(2):
        assert torch.equal(fms[b], ref[b][0])
        assert torch.equal(fvs[b], ref[b][1])
        if train:
            assert torch.equal(c_outs[b][0], ref[b][2])


@pytest.mark.parametrize("M", [1024, 200])
def test_split_upper_bounded_batch_bit_identical(device, M):
    """mgp_split_upper_f16_bounded_batch (both layers' L^-T images in one launch) writes
    the same image bits as one mgp_split_upper_f16_bounded call per layer."""
    from modulatedgps_amd import ops
    g = torch.Generator(device=device).manual_seed(3)
    Zs = [torch.randn(M, 3, device=device, generator=g) for _ in range(2)]
    var = [torch.tensor([0.8], device=device), torch.tensor([1.3], device=device)]
    ls = [torch.tensor([0.9], device=device), torch.tensor([1.4], device=device)]
    nb = ops.x6_lower_bytes(M, 1)
    imgs = [torch.zeros(nb, dtype=torch.uint8, device=device) for _ in range(2)]
    _, LinvT, _ = ops.kuu_potrf_trtri(Zs, var, ls, 1e-6, tfr_bound_images=imgs)
    ref = [ops.split_upper_x6(LinvT[b], out=imgs[b].clone(), fmt="f16", bounded=True) for b in range(2)]
    got = ops.split_upper_f16_bounded_batch(LinvT, [imgs[0].clone(), imgs[1].clone()])
    torch.cuda.synchronize()
    for b in range(2):
        assert torch.equal(got[b], ref[b])


@pytest.mark.parametrize("var", [0.1, 0.3, 0.5])
def test_kuf_f16_image_any_variance(device, var):
    """K1's split-f16 Kuf image at kernel variances that are not powers of two (the
    per-lane multiplier var * 2^e then rounds), by its own launch (mgp_rbf_kuf_f16) and
    as the side job of K3's step launches (mgp_kuu_potrf_trtri_kuf, the ELBO step's
    default; bit-identical to it): hi + lo at f32 class against float64 Kuf.
    Regression (round 6): the compiler had contracted that multiply into the hi / lo
    conversions (v_fma_mix*_f16 beside v_cvt_pk_f16_f32 of the rounded product), so lo
    did not belong to the stored hi -- at variance 0.1 the image was 2.3e-6 off
    normwise and 3e-4 of the maximum (f32 class: 2.7e-7), which made the assignment
    layer's fmean / fvar 7x less accurate than x6 (its kernel variance is 0.1) and the
    training gradient of that layer up to 12x worse than float32 autograd."""
    from modulatedgps_amd import ops
    N, M, D = 4096, 256, 8
    X, _, p = R.synthetic_problem(N, M, 1, D, 1.0, state="init", S=1)
    Z = p.pred["Z"]
    X32, Z32 = X.astype(np.float32), Z.astype(np.float32)
    Xd, Zd = _t(X32, device), _t(Z32, device)
    vt = torch.tensor([var], dtype=torch.float32, device=device)
    lt = torch.tensor([1.0], dtype=torch.float32, device=device)
    ref = R.rbf_K(Z32.astype(np.float64), X32.astype(np.float64), float(np.float32(var)), 1.0)
    # zero-filled buffers: plane 2 of a split-f16 image is never written
    img = torch.zeros(ops._lib.load().mgp_x6_cols_bytes(M, N), dtype=torch.uint8, device=device)
    ops.rbf_kuf_x6(Xd, Zd, vt, lt, out=img, fmt="f16")
    side = torch.zeros_like(img)
    ops.kuu_potrf_trtri([Zd], [vt], [lt], 1e-6, kuf=(Xd, [side], "f16"))
    torch.cuda.synchronize()
    assert torch.equal(img, side)
    bound = float(ops.image_bound(img, M, N=N).cpu())
    assert bound == pytest.approx(float(np.float32(var)))
    got = decode_cols_f16(img, M, N, bound)
    assert normwise(got, ref) < 5e-7
    assert np.abs(got - ref).max() < 2e-6 * np.abs(ref).max()


def test_conditionals_f16_any_variance(device):
    """Both layers' (fmean, fvar) of the split-f16 chain at the synthetic problem's
    kernel variances (pred 0.5, assign 0.1) against float64: the assignment layer as
    accurate as the prediction layer and as the x6 chain (round-6 regression of the
    K1 split above: assign fmean 7.6e-6 normwise at config-3 shapes, now 1.0e-6)."""
    from modulatedgps_amd import config
    N, M, K, D = 8192, 512, 4, 8
    X, _, p = R.synthetic_problem(N, M, K, D, 1.0, state="perturbed", S=1)
    errs = {}
    for fmt in ("f16", "x6"):
        old = config.expert_format()
        config.set_expert_format(fmt)
        try:
            model = build_model(p, device)
            got = [to_np(c)[:, :N] for c in model.conditionals(_t(X, device))]
        finally:
            config.set_expert_format(old)
        for name, L, gm, gv in (("pred", p.pred, got[0], got[1]), ("assign", p.assign, got[2], got[3])):
            f32 = lambda v: np.asarray(v, np.float64).astype(np.float32).astype(np.float64)
            fm, fv = R.svgp_predict_f_dedup(f32(X), f32(L["Z"]), f32(L["variance"]), f32(L["lengthscales"]),
                                            f32(L["q_mu"]), f32(L["q_sqrt"]))
            errs[fmt, name] = (normwise(gm, fm.T), normwise(gv, fv.T))
    print(errs)
    for name in ("pred", "assign"):
        for i in range(2):
            assert errs["f16", name][i] < 3e-6
            assert errs["f16", name][i] < 2.5 * errs["x6", name][i]
