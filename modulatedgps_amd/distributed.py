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


def allreduce_gradients(tensors, group=None):
    """Sum a list of gradient tensors over the group with one collective per dtype:
    the tensors are packed into a flat bucket (float32 / float64), all-reduced and
    unpacked in place.  The training step's only data-path exchange (the gradients
    of the per-shard data terms; the KL part is added after it on every rank)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return tensors
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for ts in by_dtype.values():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
        o = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[o:o + n].view_as(t))
            o += n
    return tensors


def sharded_elbo(model, X_local, Y_local, n_offset, n_total, group=None, **kw):
    """ELBO of the global batch from this rank's shard (SMGP._build_likelihood with
    the shard's global row offset and one all-reduce of the data term)."""
    pg = group if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
    if pg is not None and dist.get_world_size(pg) == 1:
        pg = None
    return model._build_likelihood(X_local, Y_local, n_offset=n_offset, n_total=n_total,
                                   process_group=pg, **kw)
