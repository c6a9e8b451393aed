"""End-to-end parity of the drop-in SMGP API (MixtureGPs.models on the MI355X
kernels) against the float64 oracle and the committed golden fixtures.

Tolerance (BASELINE.json north_star): ELBO within 1e-4 relative; predictive
mean/var and per-layer fmean/fvar within 1e-4 normwise (||a-b||/||b||), the
elementwise relative error being meaningless where fmean ~ 0."""
import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from oracle import philox
from tests.helpers import build_model, dev_noise, load_golden, normwise, params_from_golden, to_np

pytestmark = pytest.mark.gpu

CASES = ["case_demo_init", "case_demo_perturbed", "case_c1"]


@pytest.mark.parametrize("case", CASES)
def test_golden_elbo_and_predictions(device, case):
    d = load_golden(case + ".npz")
    p = params_from_golden(d)
    model = build_model(p, device)
    X = torch.as_tensor(d["X"], dtype=torch.float32, device=device)
    Y = torch.as_tensor(d["Y"], dtype=torch.float32, device=device)
    elbo = float(model._build_likelihood(X, Y, noise=dev_noise(d["z"], d["u"], device)).cpu())
    assert elbo == pytest.approx(float(d["elbo"]), rel=1e-4)
    # Philox mode against the oracle's statement of the same stream
    e2 = float(model._build_likelihood(X, Y, seed=int(d["philox_seed"])).cpu())
    assert e2 == pytest.approx(float(d["elbo_philox"]), rel=1e-4)
    # per-layer conditional
    mu_f, var_f, mu_a, var_a = model.conditionals(X)
    assert normwise(to_np(mu_f).T, d["mu_f"]) < 1e-4 or np.abs(d["mu_f"]).max() == 0
    assert normwise(to_np(var_f).T, d["var_f"]) < 1e-4
    assert normwise(to_np(var_a).T, d["var_a"]) < 1e-4
    # predictions (models.py:38-41, 85-89)
    Xt = torch.as_tensor(d["Xtest"], dtype=torch.float32, device=device)
    ym, yv = model.predict_y(Xt)
    assert tuple(ym.shape) == (1, Xt.shape[0], p.lik_variance.shape[1])
    if np.abs(d["predict_y_mean"]).max() > 0:
        assert normwise(to_np(ym), d["predict_y_mean"]) < 1e-4
    else:
        assert np.abs(to_np(ym)).max() < 1e-6
    assert normwise(to_np(yv), d["predict_y_var"]) < 1e-4
    pa = model.predict_assign(Xt)
    assert normwise(to_np(pa), d["predict_assign"]) < 1e-4


def test_golden_c2_shapes(device):
    d = load_golden("case_c2r.npz")
    gen = {k[4:]: (v.item() if v.ndim == 0 else v) for k, v in d.items() if k.startswith("gen_")}
    gen["state"] = str(gen["state"])
    X, Y, p = R.synthetic_problem(**gen)
    z, u = R.explicit_noise(25, gen["N"], gen["K"], seed=5)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    assert e == pytest.approx(float(d["elbo"]), rel=1e-4)
    ym, yv = model.predict_y(Xd[:128])
    assert normwise(to_np(ym), d["predict_y_mean"]) < 1e-4
    assert normwise(to_np(yv), d["predict_y_var"]) < 1e-4


@pytest.mark.parametrize("N,M,K,D,ls,S", [(8192, 256, 4, 2, 0.15, 25),      # BASELINE config 2
                                           (8192, 1024, 8, 8, 1.0, 25),      # config-3 shapes, N reduced
                                           (4096, 2048, 16, 16, 2.0, 25),    # config-5 shapes, N reduced
                                           (1001, 33, 2, 3, 0.8, 7)])        # ragged sizes
def test_elbo_configs(device, N, M, K, D, ls, S):
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


def test_shard_invariance_of_data_term(device):
    """Two N-shards with n_offset reproduce the unsharded Philox data term (the
    property the multi-GPU path relies on)."""
    from modulatedgps_amd import ops
    X, Y, p = R.synthetic_problem(3000, 64, 3, 2, 0.7, state="perturbed", S=5)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    Yd = torch.as_tensor(Y[:, 0], dtype=torch.float32, device=device)
    lv = model.likelihood.likelihood.variance.reshape(-1)
    full = model.conditionals(Xd)
    tot = float(ops.elbo_terms(*full, Yd, lv, 5, seed=11).cpu())
    parts = 0.0
    for lo, hi in ((0, 1234), (1234, 3000)):
        c = [t.clone() for t in model.conditionals(Xd[lo:hi])]
        parts += float(ops.elbo_terms(*c, Yd[lo:hi].contiguous(), lv, 5, seed=11, n_offset=lo).cpu())
    assert parts == pytest.approx(tot, rel=1e-6)


def test_predict_samples_parity(device):
    d = load_golden("case_demo_perturbed.npz")
    p = params_from_golden(d)
    model = build_model(p, device)
    Xt = d["Xtest"]
    S = 6
    rng = np.random.default_rng(9)
    zw = rng.standard_normal((S, Xt.shape[0], 3))
    uw = rng.uniform(1e-6, 1 - 1e-6, (S, Xt.shape[0], 3))
    zy = rng.standard_normal((S, Xt.shape[0], 3))
    sy_r, sf_r = R.predict_samples(Xt, p, S, zw, uw, zy)
    noise = [torch.as_tensor(a, dtype=torch.float32, device=device) for a in (zw, uw, zy)]
    sy, sf = model.predict_samples(torch.as_tensor(Xt, dtype=torch.float32, device=device), S,
                                   noise=noise)
    assert tuple(sy.shape) == (S, Xt.shape[0], 1)
    assert normwise(to_np(sy), sy_r) < 1e-4
    assert normwise(to_np(sf), sf_r) < 1e-4


def test_native_library_is_loaded(device):
    """The HIP library (not a fallback) is what the model runs on."""
    import modulatedgps_amd
    lib = modulatedgps_amd.library()
    assert b"gfx950" in lib.mgp_version()
    maps = open("/proc/self/maps").read()
    assert "libmgp_hip.so" in maps


@pytest.mark.parametrize("N,M,K,D,ls,S", [(1000, 25, 3, 1, 0.5, 25), (8192, 256, 4, 2, 0.15, 25),
                                           (1001, 33, 2, 3, 0.8, 7)])
def test_smgp_modified_elbo(device, N, M, K, D, ls, S):
    """SMGPModified (models.py:106-123, demo_tf2_modified.py): the MOD variant of
    K6 against the oracle's smgp_modified_elbo, same explicit noise."""
    from modulatedgps_amd.likelihoods import GaussianModified
    from modulatedgps_amd.models import SMGPModified
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    a_var = np.linspace(0.3, 0.9, K)[None, :]
    z, u = R.explicit_noise(S, N, K, seed=5)
    ref = R.smgp_modified_elbo(X, Y, p, a_var, z, u)
    base = build_model(p, device)
    model = SMGPModified(base.likelihood.likelihood, GaussianModified(variance=a_var, device=device),
                         base.pred_layer, base.assign_layer, K=K, num_samples=S, num_data=p.num_data)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    assert e == pytest.approx(ref, rel=1e-4)
    # the plain SMGP term on the same model state is different (the extra term is live)
    assert abs(float(base._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu()) - e) > 1e-3 * abs(e)


def test_conditional_experts_partition(device):
    """Expert-parallel layout: the conditionals of an expert range (K4 stats and K5
    on q_mu[:, k0:k1], q_sqrt[k0:k1]) equal those rows of the full conditional."""
    X, Y, p = R.synthetic_problem(3000, 130, 5, 3, 0.9, state="perturbed", S=4)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    for layer in (model.pred_layer, model.assign_layer):
        fm, fv = (t.clone() for t in layer.conditional_kn(Xd))
        for k0, k1 in ((0, 2), (2, 3), (3, 5)):
            em, ev = layer.conditional_experts(Xd, k0, k1)
            assert torch.equal(em[:, :3000], fm[k0:k1, :3000])
            assert torch.equal(ev[:, :3000], fv[k0:k1, :3000])


def _expert_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    from modulatedgps_amd.distributed import expert_parallel_elbo
    X, Y, p = R.synthetic_problem(2000, 64, 5, 2, 0.8, state="perturbed", S=6)
    z, u = R.explicit_noise(6, 2000, 5, seed=5)
    model = build_model(p, dev)
    e = expert_parallel_elbo(model, torch.as_tensor(X, dtype=torch.float32, device=dev), Y,
                             noise=dev_noise(z, u, dev))
    if rank == 0:
        ref = float(model._build_likelihood(torch.as_tensor(X, dtype=torch.float32, device=dev), Y,
                                            noise=dev_noise(z, u, dev)).cpu())
        q.put((float(e.cpu()), ref, R.smgp_elbo(X, Y, p, z, u)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2])
def test_expert_parallel_elbo(device, world):
    """The north_star expert layout (experts sharded over ranks, all_to_all of the
    conditionals, one scalar all-reduce) reproduces the single-process ELBO and
    the oracle.  Rehearsed with gloo, every rank on cuda:0 (the 8-GPU run uses RCCL)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_expert_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    e, ref, oracle = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    assert e == pytest.approx(ref, rel=1e-6)
    assert e == pytest.approx(oracle, rel=1e-4)


def test_cholesky_failure_raises(device):
    """A non-SPD Kuu (duplicated inducing points, zero jitter) raises MGPLinAlgError
    where the reference raises InvalidArgumentError from base_conditional
    (models.py:141): at run_adam's ELBO readback and in the predict_* methods."""
    from modulatedgps_amd import config
    from modulatedgps_amd._lib import MGPLinAlgError
    from utils.data import Dataset
    from utils.training_utils import run_adam
    X, Y, p = R.synthetic_problem(500, 20, 3, 1, 0.5, state="perturbed", S=5)
    p.pred["Z"][7] = p.pred["Z"][3]                   # two identical rows: Kuu singular
    old = config.default_jitter()
    config.set_default_jitter(0.0)
    try:
        model = build_model(p, device)
        Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
        model._build_likelihood(Xd, Y)                 # asynchronous: no raise here
        assert int(model.last_info.cpu()[0]) > 0
        with pytest.raises(MGPLinAlgError):
            model.check_linalg()
        with pytest.raises(MGPLinAlgError):
            model.predict_y(Xd)
        with pytest.raises(MGPLinAlgError):
            model.predict_samples(Xd, S=2)
        it = iter(Dataset.from_tensor_slices((X, Y)).shuffle(500, seed=0).batch(100).repeat())
        with pytest.raises(MGPLinAlgError):
            run_adam(model, 10, it, 0.01)
    finally:
        config.set_default_jitter(old)


def test_default_jitter_reaches_sampling(device):
    """set_default_jitter changes both Kuu's jitter and the reparameterisation
    jitter of W_dist / predict_samples (utils.py:26-27 reads default_jitter())."""
    from modulatedgps_amd import config
    X, Y, p = R.synthetic_problem(700, 25, 3, 1, 0.5, state="perturbed", S=6)
    z, u = R.explicit_noise(6, 700, 3, seed=5)
    old, old_r = config.default_jitter(), R.JITTER
    try:
        config.set_default_jitter(1e-3)
        R.JITTER = 1e-3
        ref = R.smgp_elbo(X, Y, p, z, u)
        model = build_model(p, device)
        Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
        e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
        assert e == pytest.approx(ref, rel=1e-4)
        rng = np.random.default_rng(9)
        zw, uw, zy = rng.standard_normal((4, 700, 3)), rng.uniform(1e-6, 1 - 1e-6, (4, 700, 3)), \
            rng.standard_normal((4, 700, 3))
        sy_r, sf_r = R.predict_samples(X, p, 4, zw, uw, zy)
        noise = [torch.as_tensor(a, dtype=torch.float32, device=device) for a in (zw, uw, zy)]
        sy, sf = model.predict_samples(Xd, 4, noise=noise)
        assert normwise(sf, sf_r) < 1e-4 and normwise(sy, sy_r) < 1e-4
    finally:
        config.set_default_jitter(old)
        R.JITTER = old_r


def test_elbo_returns_fresh_tensors(device):
    """Each evaluation returns its own tensor (kept values do not alias the buffers)."""
    X, Y, p = R.synthetic_problem(600, 20, 3, 1, 0.5, state="perturbed", S=5)
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    vals = [model.elbo((Xd, Y)) for _ in range(3)]     # fresh Philox noise per call
    host = [float(v.cpu()) for v in vals]
    assert len(set(host)) == 3
    e, _ = model.elbo_and_grad(Xd, Y)
    assert float(vals[0].cpu()) == host[0] and e.data_ptr() != vals[-1].data_ptr()
