"""CPU tests of the N-sharded data-parallel path (world_size 2, gloo).

The HIP kernels need a GPU, so the per-shard compute here is the float64
oracle; what is tested is the host logic the multi-GPU bench relies on: the
row partition, shard invariance of the Philox noise keyed by the global row,
and that one all-reduce of the per-shard data-term sums reproduces the
single-process ELBO."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from modulatedgps_amd.distributed import allreduce_data_term, shard_rows


@pytest.mark.parametrize("n,world", [(10, 3), (65536, 8), (7, 8), (1001, 2)])
def test_shard_rows_partition(n, world):
    spans = [shard_rows(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data_term_sum(X, Y, p, n_global, seed):
    from oracle import cpu_ref as R
    from oracle import philox
    K = p.lik_variance.shape[1]
    z = philox.noise_normal(seed, p.S, n_global, K)
    u = philox.noise_uniform(seed, p.S, n_global, K)
    mu_a, var_a = R.svgp_predict_f_dedup(X, p.assign["Z"], p.assign["variance"], p.assign["lengthscales"],
                                         p.assign["q_mu"], p.assign["q_sqrt"])
    mu_f, var_f = R.svgp_predict_f_dedup(X, p.pred["Z"], p.pred["variance"], p.pred["lengthscales"],
                                         p.pred["q_mu"], p.pred["q_sqrt"])
    W = R.assignment_weights(mu_a[None], var_a[None], z, u)
    return float(np.sum(R.e_log_p_y(mu_f[None], var_f[None], Y, p.lik_variance, W, p.S)))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cpu_ref as R
    N = 300
    X, Y, p = R.synthetic_problem(N, 12, 3, 2, 0.6, state="perturbed", S=4)
    lo, hi = shard_rows(N, rank, world)
    part = _data_term_sum(X[lo:hi], Y[lo:hi], p, np.arange(lo, hi), seed=42)
    t = torch.tensor([part], dtype=torch.float64)
    allreduce_data_term(t)
    if rank == 0:
        full = _data_term_sum(X, Y, p, np.arange(N), seed=42)
        kl = R.gauss_kl_white(p.pred["q_mu"], p.pred["q_sqrt"]) + \
            R.gauss_kl_white(p.assign["q_mu"], p.assign["q_sqrt"])
        elbo_dp = float(t.item()) / N - kl / p.num_data
        from oracle import philox
        z = philox.noise_normal(42, p.S, np.arange(N), 3)
        u = philox.noise_uniform(42, p.S, np.arange(N), 3)
        elbo_ref = R.smgp_elbo(X, Y, p, z, u)
        q.put((float(t.item()), full, elbo_dp, elbo_ref))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_two_rank_allreduce_reproduces_full_elbo(world):
    """One float64 all-reduce of the per-shard data-term sums == the single-process
    ELBO, at world 2 and at the north_star's 8 ranks (uneven 300 / 8 shards)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    reduced, full, elbo_dp, elbo_ref = res
    assert reduced == pytest.approx(full, rel=1e-12)
    assert elbo_dp == pytest.approx(elbo_ref, rel=1e-12)


def _grad_worker(rank, world, port, q):
    """Data-parallel training-step gradient: each rank differentiates its shard's
    data term (scaled by 1 / N_total) with the float64 autograd oracle, the
    gradients go through modulatedgps_amd.distributed.allreduce_gradients_async in
    the per-layer buckets SMGP.elbo_and_grad issues (likelihood + pred layer, then
    assign layer, both in flight before either is waited for), then every rank adds
    the KL gradient.  Rank 0 compares with the single-process gradient."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from modulatedgps_amd.distributed import allreduce_gradients_async
    from oracle import cpu_ref as R
    from oracle import grad_ref as GR
    N = 240
    X, Y, p = R.synthetic_problem(N, 10, 3, 2, 0.7, state="perturbed", S=3)
    z, u = R.explicit_noise(p.S, N, 3, seed=11)
    t64 = lambda a: torch.tensor(np.asarray(a, np.float64))

    def leaves():
        pred, assign, lik = GR.params_from_oracle(p)
        return pred, assign, lik

    def grads_of(pred, assign, lik):
        out = [lik.grad]
        for L in (pred, assign):
            out += [L[k].grad for k in GR.LAYER_KEYS]
        return out

    # this rank's shard
    lo, hi = shard_rows(N, rank, world)
    pred, assign, lik = leaves()
    mu_f, var_f, _ = GR.layer_conditional(t64(X[lo:hi]), pred)
    mu_a, var_a, _ = GR.layer_conditional(t64(X[lo:hi]), assign)
    dt = GR.data_term(mu_f, var_f, mu_a, var_a, t64(Y[lo:hi]), lik, t64(z[:, lo:hi]), t64(u[:, lo:hi]))
    (dt / N).backward()
    g = [t.clone() for t in grads_of(pred, assign, lik)]
    pending = [allreduce_gradients_async(g[:6]), allreduce_gradients_async(g[6:])]
    for pb in pending:
        pb.wait()
    # KL part, added locally after the reduction
    pred2, assign2, lik2 = leaves()
    kl = GR.gauss_kl_white(pred2["q_mu"], pred2["q_sqrt"]) + GR.gauss_kl_white(assign2["q_mu"], assign2["q_sqrt"])
    (-kl / p.num_data).backward()
    for i, L in enumerate((pred2, assign2)):
        for j, k in enumerate(GR.LAYER_KEYS):
            if L[k].grad is not None:
                g[1 + 5 * i + j] = g[1 + 5 * i + j] + L[k].grad
    if rank == 0:
        pr, asg, lk = leaves()
        GR.elbo(t64(X), t64(Y), pr, asg, lk, t64(z), t64(u), p.num_data).backward()
        ref = grads_of(pr, asg, lk)
        q.put([float((a - b).abs().max() / (b.abs().max() + 1e-300)) for a, b in zip(g, ref)])
    dist.destroy_process_group()


def test_two_rank_gradient_allreduce_reproduces_full_gradient():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    errs = q.get(timeout=180)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert max(errs) < 1e-10, errs


def _a2a_worker(rank, world, port, q, K=5):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from modulatedgps_amd.distributed import redistribute_experts
    C, N = 4, 37
    counts = [b - a for a, b in (shard_rows(K, r, world) for r in range(world))]
    k0, k1 = shard_rows(K, rank, world)
    k = torch.arange(k0, k1, dtype=torch.float32)[:, None, None]
    c = torch.arange(C, dtype=torch.float32)[None, :, None]
    n = torch.arange(N, dtype=torch.float32)[None, None, :]
    local = 1000 * k + 100 * c + n
    mine = redistribute_experts(local, counts, N)
    lo, hi = shard_rows(N, rank, world)
    kk = torch.arange(K, dtype=torch.float32)[:, None, None]
    ref = 1000 * kk + 100 * c + torch.arange(lo, hi, dtype=torch.float32)[None, None, :]
    q.put((rank, bool(torch.equal(mine, ref)), tuple(mine.shape)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,K", [(2, 5), (3, 5), (8, 8)])
def test_expert_layout_redistribution(world, K):
    """Expert-parallel layout (north_star: experts sharded over GPUs): the exchange
    that moves every expert's conditionals to the rank owning each point slice
    (all_to_all on RCCL, point-to-point on gloo), including a rank with fewer
    experts than another (K = 5), and the north_star's exact c4 partition: K = 8
    experts over 8 ranks, one expert each (counts [1] * 8), N = 37 in 8 slices."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_a2a_worker, args=(r, world, port, q, K)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    assert all(ok for _, ok, _ in res), res
