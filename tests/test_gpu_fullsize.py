"""Parity at the BASELINE workloads' full sizes.

* c3 (N = 65536, M = 1024, K = 8, D = 8, S = 25): the whole ELBO, both layers'
  fmean / fvar and predict_y against the float64 oracle at the north_star gate
  (ELBO 1e-4 relative, the rest 1e-4 normwise), in every forward image format
  (split-bf16 x6, split-f16, split-f16 with e4m3 cross terms).
* c5 per rank (the 8-GPU N-shard of N = 262144: N = 32768, M = 2048, K = 16,
  D = 16, lengthscale 2): the default format at the same gate, and the 1-plane
  "bf16 mixed" K5 mode at its stated looser tolerance (measured,
  not gated at 1e-4; the bound below is its measured error with 2x margin).
* c4 (c3's N sharded over ranks, one RCCL all-reduce of the data term): two
  ranks on one GPU (gloo, the box has one GPU) through
  SMGP._build_likelihood(process_group=...), against the single-process ELBO
  and the oracle, with explicit noise and with in-kernel Philox noise.
The oracle runs once per module (about 4 s at c3, 20-40 s at c5 per rank on the
box's host cores)."""
import socket

import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from tests.helpers import build_model, dev_noise, normwise, to_np

pytestmark = pytest.mark.gpu

C3 = (65536, 1024, 8, 8, 1.0, 25)
C5_RANK = (32768, 2048, 16, 16, 2.0, 25)


def _problem(cfg):
    N, M, K, D, ls, S = cfg
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    ref, parts = R.smgp_elbo(X, Y, p, z, u, return_parts=True)
    return X, Y, p, z, u, ref, parts


@pytest.fixture(scope="module")
def c3():
    return _problem(C3)


@pytest.fixture(scope="module")
def c5_rank():
    return _problem(C5_RANK)


@pytest.fixture
def image_mode(request):
    from modulatedgps_amd import config
    old = (config.expert_format(), config.expert_cross(), config.expert_planes())
    fmt, cross, planes = request.param
    config.set_expert_format(fmt)
    config.set_expert_cross(cross)
    config.set_expert_planes(planes)
    yield request.param
    config.set_expert_format(old[0])
    config.set_expert_cross(old[1])
    config.set_expert_planes(old[2])


def _check_full(device, prob, tol_elbo, tol_norm, with_predict=True):
    X, Y, p, z, u, ref, parts = prob
    model = build_model(p, device)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    mu_f, var_f, mu_a, var_a = model.conditionals(Xd)
    errs = {"elbo": abs(e - ref) / abs(ref)}
    for name, t in (("mu_f", mu_f), ("var_f", var_f), ("mu_a", mu_a), ("var_a", var_a)):
        errs[name] = normwise(to_np(t).T, parts[name])
    if with_predict:
        ym, yv = model.predict_y(Xd)
        my, vy = R.gaussian_predict_mean_and_var(parts["mu_f"], parts["var_f"], p.lik_variance)
        errs["predict_y_mean"] = normwise(ym[0], my)
        errs["predict_y_var"] = normwise(yv[0], vy)
    print({k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["elbo"] < tol_elbo
    for k, v in errs.items():
        if k != "elbo":
            assert v < tol_norm, (k, v)
    return errs


@pytest.mark.timeout(300)
@pytest.mark.parametrize("image_mode", [("x6", "f16", 3), ("f16", "f16", 3), ("f16", "f8", 3)],
                         ids=["x6", "f16", "f16x8"], indirect=True)
def test_c3_full_size(device, c3, image_mode):
    _check_full(device, c3, 1e-4, 1e-4)


@pytest.mark.timeout(600)
def test_c5_per_rank_full_size(device, c5_rank):
    """c5's per-rank shape in the default (split-f16) chain at the north_star gate."""
    _check_full(device, c5_rank, 1e-4, 1e-4)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("image_mode", [("x6", "f16", 1)], ids=["bf16-mixed"], indirect=True)
def test_c5_per_rank_bf16_mixed(device, c5_rank, image_mode):
    """c5's "bf16 mixed" K5 (one bf16 plane per operand; K1/K4/K3 unchanged):
    SURVEY §8d states a looser, measured tolerance.  Measured here: fvar 2e-3
    normwise at c3 (bench k5_modes.planes1); the bound is 1e-2 on the
    conditionals and 1e-3 relative on the ELBO."""
    errs = _check_full(device, c5_rank, 1e-3, 1e-2, with_predict=False)
    assert errs["mu_f"] < 1e-4 and errs["mu_a"] < 1e-4   # fmean comes from K4 (x6), not K5


# --------------------------------------------------------------------------- c4
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _c4_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    from modulatedgps_amd.distributed import shard_rows, sharded_elbo
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    N, M, K, D, ls, S = C3
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    lo, hi = shard_rows(N, rank, world)
    model = build_model(p, dev, seed=7)
    Xl = torch.as_tensor(X[lo:hi], dtype=torch.float32, device=dev)
    e_noise = sharded_elbo(model, Xl, Y[lo:hi], lo, N, noise=dev_noise(z[:, lo:hi], u[:, lo:hi], dev))
    e_philox = sharded_elbo(model, Xl, Y[lo:hi], lo, N, seed=1234)
    q.put((rank, float(e_noise.cpu()), float(e_philox.cpu())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_c4_sharded_elbo(device, c3):
    """c4: c3's N split over two ranks (gloo rehearsal on one GPU; the 8-GPU run
    uses RCCL with the same code path).  Every rank's ELBO equals the
    single-process ELBO (explicit noise: rel 1e-6; Philox keyed by the global
    row: rel 1e-6) and the oracle (1e-4)."""
    import torch.multiprocessing as mp
    X, Y, p, z, u, ref, _ = c3
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted(q.get(timeout=500) for _ in range(world))
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    model = build_model(p, device, seed=7)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    single_noise = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    single_philox = float(model._build_likelihood(Xd, Y, seed=1234).cpu())
    print("c4 ranks:", res, "single:", single_noise, single_philox, "oracle:", ref)
    for _, e_noise, e_philox in res:
        assert e_noise == pytest.approx(single_noise, rel=1e-6)
        assert e_noise == pytest.approx(ref, rel=1e-4)
        assert e_philox == pytest.approx(single_philox, rel=1e-6)
