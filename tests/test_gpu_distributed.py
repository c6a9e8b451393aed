"""Multi-process paths on the GPU (BASELINE c4).

The box has one GPU, so multi-rank runs are gloo rehearsals with every rank on
cuda:0 (RCCL refuses two ranks on one device); the RCCL code path itself is
exercised by a one-rank "nccl" group, whose collectives run through RCCL on the
device.

* c4 in the north_star's expert layout at its full config (N = 65536, M = 1024,
  K = 8, D = 8): experts sharded over two ranks, one all_to_all of the
  conditionals, one scalar all-reduce -- against the float64 oracle (1e-4) and
  the single-process ELBO (1e-6).
* The training step's data-parallel gradient (SMGP.elbo_and_grad with a
  process group: each rank differentiates its N-shard, one bucketed all-reduce)
  at BASELINE c2, against the single-process gradient.
"""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from tests.helpers import build_model, dev_noise, normwise

pytestmark = pytest.mark.gpu

C3 = (65536, 1024, 8, 8, 1.0, 25)
C2 = (8192, 256, 4, 2, 0.15, 25)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(target, world, extra=()):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *extra)) for r in range(world)]
    for pr in procs:
        pr.start()
    return procs, q


def _join(procs):
    for pr in procs:
        pr.join(timeout=180)
        assert pr.exitcode == 0


def _init(rank, world, port, backend="gloo"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return dist


# --------------------------------------------------------------------------- c4, expert layout
def _c4_expert_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    from modulatedgps_amd.distributed import expert_parallel_elbo
    dev = torch.device("cuda", 0)
    N, M, K, D, ls, S = C3
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    model = build_model(p, dev, seed=7)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=dev)
    e_noise = float(expert_parallel_elbo(model, Xd, Y, noise=dev_noise(z, u, dev)).cpu())
    e_philox = float(expert_parallel_elbo(model, Xd, Y, seed=4321).cpu())
    q.put((rank, e_noise, e_philox))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 8])
def test_c4_expert_layout_full_size(device, world):
    """BASELINE c4 as north_star states it (the K = 8 experts sharded over the
    ranks): 4 + 4 on two ranks, and the exact north_star partition -- one expert
    per rank on 8 ranks (counts [1] * 8 in the all_to_all, 8 point slices) -- at
    N = 65536, M = 1024, D = 8 (gloo ranks sharing cuda:0 on the one-GPU box)."""
    N, M, K, D, ls, S = C3
    procs, q = _spawn(_c4_expert_worker, world)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    ref = R.smgp_elbo(X, Y, p, z, u)
    res = sorted(q.get(timeout=800) for _ in range(world))
    _join(procs)
    assert len(res) == world
    model = build_model(p, device, seed=7)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    single_noise = float(model._build_likelihood(Xd, Y, noise=dev_noise(z, u, device)).cpu())
    single_philox = float(model._build_likelihood(Xd, Y, seed=4321).cpu())
    print("c4 expert layout:", res, "single:", single_noise, single_philox, "oracle:", ref)
    for _, e_noise, e_philox in res:
        assert e_noise == pytest.approx(ref, rel=1e-4)
        assert e_noise == pytest.approx(single_noise, rel=1e-6)
        assert e_philox == pytest.approx(single_philox, rel=1e-6)


# --------------------------------------------------------------------------- training gradient, N-sharded
def _grad_worker(rank, world, port, q):
    dist = _init(rank, world, port)
    from modulatedgps_amd.distributed import shard_rows
    dev = torch.device("cuda", 0)
    N, M, K, D, ls, S = C2
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    lo, hi = shard_rows(N, rank, world)
    model = build_model(p, dev, seed=7)
    Xl = torch.as_tensor(X[lo:hi], dtype=torch.float32, device=dev)
    e, g = model.elbo_and_grad(Xl, Y[lo:hi], noise=dev_noise(z[:, lo:hi], u[:, lo:hi], dev), n_offset=lo,
                               n_total=N, process_group=dist.group.WORLD)
    e2, g2 = model.elbo_and_grad(Xl, Y[lo:hi], seed=99, n_offset=lo, n_total=N, process_group=dist.group.WORLD)
    q.put((rank, float(e.cpu()), {k: v.double().cpu().numpy() for k, v in g.items()}, float(e2.cpu()),
           {k: v.double().cpu().numpy() for k, v in g2.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_rank_gradient_c2(device):
    """Data-parallel training step: two ranks' sharded gradients, after the one
    bucketed all-reduce, equal the single-process gradient of the whole batch
    (explicit noise and Philox keyed by the global row)."""
    N, M, K, D, ls, S = C2
    procs, q = _spawn(_grad_worker, 2)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    model = build_model(p, device, seed=7)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
    e1, g1 = model.elbo_and_grad(Xd, Y, noise=dev_noise(z, u, device))
    e1p, g1p = model.elbo_and_grad(Xd, Y, seed=99)
    res = sorted((q.get(timeout=500) for _ in range(2)), key=lambda r: r[0])
    _join(procs)
    single = ({k: v.double().cpu().numpy() for k, v in g1.items()},
              {k: v.double().cpu().numpy() for k, v in g1p.items()})
    for _, e, g, ep, gp in res:
        assert e == pytest.approx(float(e1.cpu()), rel=1e-6)
        assert ep == pytest.approx(float(e1p.cpu()), rel=1e-6)
        errs = {k: max(normwise(g[k], single[0][k]), normwise(gp[k], single[1][k])) for k in single[0]}
        print({k: f"{v:.1e}" for k, v in errs.items()})
        for k, err in errs.items():   # reduction order only (f32 shard sums vs split-K of one pass)
            assert err < 1e-4, (k, err)


# --------------------------------------------------------------------------- RCCL
def _rccl_worker(rank, world, port, q):
    dist = _init(rank, world, port, backend="nccl")
    from modulatedgps_amd.distributed import expert_parallel_elbo
    dev = torch.device("cuda", 0)
    N, M, K, D, ls, S = 4096, 128, 4, 3, 0.8, 9
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    model = build_model(p, dev, seed=7)
    Xd = torch.as_tensor(X, dtype=torch.float32, device=dev)
    noise = dev_noise(z, u, dev)
    plain = float(model._build_likelihood(Xd, Y, noise=noise).cpu())
    via = float(model._build_likelihood(Xd, Y, noise=noise, process_group=dist.group.WORLD).cpu())
    expert = float(expert_parallel_elbo(model, Xd, Y, noise=noise).cpu())
    # the training step's per-layer gradient buckets through RCCL (async, overlapped
    # with the next layer's backward) against the step without a process group
    e0, g0 = model.elbo_and_grad(Xd, Y, noise=noise)
    g0 = {k: v.double().cpu() for k, v in g0.items()}
    e1, g1 = model.elbo_and_grad(Xd, Y, noise=noise, process_group=dist.group.WORLD)
    gdiff = max(float((v.double().cpu() - g0[k]).abs().max() / (g0[k].abs().max() + 1e-30)) for k, v in g1.items())
    q.put((dist.get_backend(), plain, via, expert, R.smgp_elbo(X, Y, p, z, u), float(e0.cpu()), float(e1.cpu()),
           gdiff))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_collectives_on_device(device):
    """The ELBO's all-reduce, the expert layout's all_to_all and the training step's
    gradient buckets through RCCL (backend "nccl") on device tensors, one rank."""
    procs, q = _spawn(_rccl_worker, 1)
    backend, plain, via, expert, ref, e0, e1, gdiff = q.get(timeout=280)
    _join(procs)
    assert backend == "nccl"
    assert e1 == pytest.approx(e0, rel=1e-7) and gdiff < 1e-6
    assert via == pytest.approx(plain, rel=1e-7) and expert == pytest.approx(plain, rel=1e-6)
    assert plain == pytest.approx(ref, rel=1e-4)
