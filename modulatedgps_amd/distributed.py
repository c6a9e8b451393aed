"""Data-parallel SMGP ELBO over N (one process per GPU, torch.distributed).

The ELBO's data term is a mean over independent data points
(models.py:66-67,76), so the path shards over N with no data-path exchange:
every rank evaluates the conditional and the Monte-Carlo term for its own
contiguous row shard, and ONE all-reduce (sum) of the data-term scalar
(RCCL over xGMI with backend "nccl"; gloo in the CPU tests) produces the
global ELBO on every rank.  Kuu, its Cholesky and the KL terms are replicated
(M^3/3 and K M^2 work, negligible).  The Philox noise is keyed by the GLOBAL
row index (n_offset), so results are invariant to the number of ranks up to
the order of the floating-point sum.
"""
import os

import torch
import torch.distributed as dist


def shard_rows(n_total, rank, world):
    """Contiguous, balanced [lo, hi) row range of `rank` (sizes differ by <= 1)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("invalid rank/world")
    base, rem = divmod(int(n_total), int(world))
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's environment.
    Returns (rank, world, local_rank); a no-op single process when WORLD_SIZE is unset."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, **kw)
    return rank, world, local


def allreduce_data_term(t, group=None):
    """Sum a data-term partial (device or host tensor) over the group in place."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class PendingBucket:
    """An all-reduce of one gradient bucket in flight (allreduce_gradients_async);
    wait() orders the current stream after it and unpacks the sums in place."""

    def __init__(self, works, packs):
        self._works, self._packs = works, packs

    def wait(self):
        for w in self._works:
            w.wait()
        for flat, ts in self._packs:
            o = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[o:o + n].view_as(t))
                o += n
        self._works, self._packs = [], []


def allreduce_gradients_async(tensors, group=None):
    """Start the sum of a list of gradient tensors over the group, one collective per
    dtype: the tensors are packed into a flat bucket (float32 / float64) on the
    current stream and all-reduced asynchronously (RCCL runs it on its own stream,
    after the bucket is packed), so the caller's next kernels -- the other layer's
    backward -- overlap it.  The tensors must not change until wait()."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return PendingBucket([], [])
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    works, packs = [], []
    for ts in by_dtype.values():
        flat = torch.cat([t.reshape(-1) for t in ts])
        works.append(dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group, async_op=True))
        packs.append((flat, ts))
    return PendingBucket(works, packs)


def allreduce_gradients(tensors, group=None):
    """Sum a list of gradient tensors over the group (allreduce_gradients_async, then
    wait).  The training step's only data-path exchange: the gradients of the
    per-shard data terms (the KL part is added after it on every rank)."""
    allreduce_gradients_async(tensors, group).wait()
    return tensors


def redistribute_experts(local, counts, n_total, group=None):
    """Expert-parallel exchange: `local` [K_r, C, n_total] holds this rank's experts
    over every point; returns [K, C, n_me], all experts (in rank order) on this
    rank's point slice shard_rows(n_total, rank, world).  One all_to_all (RCCL);
    point-to-point sends with gloo, which has no all_to_all."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    spans = [shard_rows(n_total, r, world) for r in range(world)]
    C = local.shape[1]
    lo, hi = spans[rank]
    sends = [local[:, :, a:b].contiguous() for a, b in spans]
    recvs = [torch.empty((counts[r], C, hi - lo), dtype=local.dtype, device=local.device) for r in range(world)]
    if dist.get_backend(group) == "gloo":   # CPU rehearsal path (gloo moves host tensors)
        cs = [t.cpu() for t in sends]
        cr = [torch.empty(t.shape, dtype=t.dtype) for t in recvs]
        ops_ = []
        for r in range(world):
            if r == rank:
                cr[r].copy_(cs[r])
                continue
            if cs[r].numel():
                ops_.append(dist.P2POp(dist.isend, cs[r], r, group))
            if cr[r].numel():
                ops_.append(dist.P2POp(dist.irecv, cr[r], r, group))
        if ops_:
            for req in dist.batch_isend_irecv(ops_):
                req.wait()
        for r in range(world):
            recvs[r].copy_(cr[r])
    else:
        dist.all_to_all(recvs, sends, group=group)
    return torch.cat(recvs, 0)


def expert_parallel_elbo(model, X, Y, group=None, seed=None, noise=None):
    """SMGP ELBO in the north_star's expert layout: every rank holds
    all N points and computes the conditionals of its own experts
    (shard_rows(K, rank, world)) for both layers; one all_to_all moves each
    expert's (fmean, fvar) of both layers to the rank owning that point slice;
    K6 runs on the slice (the softmax over K and the logsumexp over S need all
    experts of a point); ONE all-reduce of the data-term scalar, then the
    replicated KL.  noise: optional explicit (z, u) [S, N, K] device tensors."""
    from . import ops
    pg = group if group is not None else dist.group.WORLD
    world = dist.get_world_size(pg)
    rank = dist.get_rank(pg)
    X = model.pred_layer.kernel._x(X)
    N = X.shape[0]
    K = model.K
    k0, k1 = shard_rows(K, rank, world)
    counts = [b - a for a, b in (shard_rows(K, r, world) for r in range(world))]
    dev = X.device
    local = torch.zeros((k1 - k0, 4, N), dtype=torch.float32, device=dev)
    if k1 > k0:
        for i, layer in enumerate((model.pred_layer, model.assign_layer)):
            fm, fv = layer.conditional_experts(X, k0, k1)
            local[:, 2 * i] = fm[:, :N]
            local[:, 2 * i + 1] = fv[:, :N]
    mine = redistribute_experts(local, counts, N, pg)            # [K, 4, n]
    lo, hi = shard_rows(N, rank, world)
    n = hi - lo
    cond = ops.padded(4 * K, n, dev)
    for c in range(4):
        cond[c * K:(c + 1) * K].copy_(mine[:, c])
    Yd = torch.as_tensor(Y, dtype=torch.float32, device=dev).reshape(-1)[lo:hi].contiguous()
    if seed is None and noise is None:
        seed = model.next_seed()
    nz = None
    if noise is not None:
        nz = (noise[0][:, lo:hi].contiguous(), noise[1][:, lo:hi].contiguous())
    mc = model._mc_eps()
    lik_var = None if mc is not None else model.likelihood.likelihood.variance.reshape(-1)
    data = ops.elbo_terms(cond[0:K], cond[K:2 * K], cond[2 * K:3 * K], cond[3 * K:4 * K], Yd, lik_var,
                          model.num_samples, 1e-2, noise=nz, seed=seed or 0, n_offset=lo,
                          assign_lik_var=model._assign_lik_var(), multiclass_eps=mc)
    allreduce_data_term(data, pg)
    kl = torch.cat([model.pred_layer.prior_kl(), model.assign_layer.prior_kl()])
    num_data = model.num_data if model.num_data is not None else N
    elbo, _ = ops.elbo_combine(data, kl[0:1], kl[1:2], N, num_data)
    return elbo


def sharded_elbo(model, X_local, Y_local, n_offset, n_total, group=None, **kw):
    """ELBO of the global batch from this rank's shard (SMGP._build_likelihood with
    the shard's global row offset and one all-reduce of the data term)."""
    pg = group if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    if pg is not None and dist.get_world_size(pg) == 1:
        pg = None
    return model._build_likelihood(X_local, Y_local, n_offset=n_offset, n_total=n_total,
                                   process_group=pg, **kw)
