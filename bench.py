#!/usr/bin/env python
"""Benchmark of the SMGP ELBO hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

A step is one full SMGP ELBO evaluation (SMGP._build_likelihood,
MixtureGPs/models.py:69-79: both SVGP layers, S = 25 Monte-Carlo samples,
both KLs) over one batch of synthetic input already resident in HBM, with
fresh in-kernel Philox noise per step.  Workload (N = 1): BASELINE config 3,
N = 65536, M = 1024, K = 8, D = 8, fp32, per GPU.  Multi-GPU: data-parallel
over N, one process per GPU (`--gpus N` without torchrun starts the N ranks
itself).  `--scaling strong` (default): BASELINE config c4, c3's N = 65536
split over the ranks (N / world points per GPU, one whole-config ELBO per
step); `--scaling weak`: every rank holds its own 65536-point shard of the
global batch.  `--config c4r` is c4's per-rank shape (N = 8192) on one GPU,
the single-GPU bound of the 8-GPU point.  Kuu/Cholesky/KL are replicated; ONE RCCL
all-reduce of the data-term scalar per step.  `--layout expert`: the
north_star layout (experts sharded, one all_to_all).  Timing: W warmup steps,
then the K timed steps as `--repeats` blocks (default 5 x 50), each bracketed by
barrier + synchronize, max over ranks; `value` = the median block rate in
units of whole-config evaluations (weak: world_size evaluations per step).

Rank 0 prints ONE JSON line (see README/DESIGN for the fields).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (N per GPU, M, K, D, lengthscale, S)
    "c2": (8192, 256, 4, 2, 0.15, 25),
    "c3": (65536, 1024, 8, 8, 1.0, 25),
    "c4r": (8192, 1024, 8, 8, 1.0, 25),   # c4's per-rank shard: c3's N over 8 GPUs
    "c5": (262144, 2048, 16, 16, 2.0, 25),
}
PEAK_F32_MFMA = 157.3e12      # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_BF16_MFMA = 2.5e15       # MI355X_MICROARCH.md: Peak BF16 MFMA, dense
PEAK_X6 = PEAK_BF16_MFMA / 6  # split-bf16 K4/K5: 6 bf16 products per f32 product
PEAK_F64 = 78.6e12            # FP64 vector/matrix (half the f32 rate)
PEAK_HBM = 8.0e12             # HBM3E spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=250,
                    help="timed steps in total, run as --repeats contiguous blocks (default 5 x 50)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=5,
                    help="the timed steps are split into this many blocks, each bracketed by barrier + "
                         "synchronize; value = the median block rate (SURVEY §8d: median of 5 repeats)")
    ap.add_argument("--scaling", default="strong", choices=("weak", "strong"),
                    help="multi-GPU data layout: 'strong' (the default) = BASELINE config c4, the config's N "
                         "sharded over the ranks (N / world per GPU); 'weak' = N points per GPU")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--planes", type=int, default=3, choices=(1, 2, 3),
                    help="bf16 planes per operand in K5 (3: f32-accurate x6, the default; 2 / 1: the "
                         "'bf16 mixed' modes of BASELINE config 5, reported with their measured tolerance)")
    ap.add_argument("--format", default=None, choices=("x6", "f16"),
                    help="image format of the forward K4 -> K5 hand-off: x6 (split-bf16, 6 products) or f16 "
                         "(split-f16, 3 products, 22-bit operands); default: modulatedgps_amd.config")
    ap.add_argument("--cross", default=None, choices=("f16", "f8"),
                    help="split-f16 K5: cross terms a_hi b_lo + a_lo b_hi on f16 (3 f16 products) or on one "
                         "e4m3 MFMA per two k-steps (f16x8); default: modulatedgps_amd.config")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-modes", action="store_true", help="skip the reduced-plane K5 side measurements")
    ap.add_argument("--no-train", action="store_true", help="skip the training-step (ELBO + gradient + Adam) leg")
    ap.add_argument("--layout", default="data", choices=("data", "expert"),
                    help="multi-GPU layout: 'data' shards N (weak scaling, the default); 'expert' shards the "
                         "K experts over the ranks on a fixed N (the north_star layout, strong scaling)")
    ap.add_argument("--cpu-sample", type=int, nargs=2, default=(8192, 65536),
                    help="two N sizes of the CPU oracle sample (linear fit in N; the full N "
                         "is timed directly when it is one of them)")
    return ap.parse_args()


def timed_blocks(step, steps, repeats, barrier, world, device, timing=None):
    """Run `steps` timed steps as `repeats` contiguous blocks, each bracketed by a
    barrier + torch.cuda.synchronize() on both sides; every block's wall time is the
    max over ranks.  Returns (per-block (steps, seconds) list, last step's result)."""
    repeats = max(1, min(repeats, steps))
    sizes = [steps // repeats + (1 if r < steps % repeats else 0) for r in range(repeats)]
    blocks, out = [], None
    for n in sizes:
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            out = step(timing)
        torch.cuda.synchronize()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=device, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            el = float(t.item())
        blocks.append((n, el))
    return blocks, out


def median_rate(blocks, world):
    """Median over blocks of world * steps / seconds, and its ms per step."""
    rates = sorted(world * n / el for n, el in blocks)
    med = float(np.median(rates))
    return med, world / med * 1e3, [round(r, 2) for r in rates]


def launch_ranks(args):
    """`python bench.py --gpus N` without torchrun: start N ranks as child processes
    (torch.distributed.run, 127.0.0.1 rendezvous, one GPU per rank) before anything
    touches the GPU, and exit with their status.  Fails if fewer than N devices are
    visible (device_count() does not initialise the GPU on this image), unless the
    MGP_BENCH_SHARE_GPU=1 rehearsal puts every rank on cuda:0."""
    import socket
    import subprocess
    share = os.environ.get("MGP_BENCH_SHARE_GPU") == "1"
    have = torch.cuda.device_count()
    if not share and have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {have} device(s) visible", file=sys.stderr)
        sys.exit(2)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def synthetic(cfg, rank, device):
    """SURVEY §8(d) synthetic inputs: X ~ N(0, I_D) (per-rank shard), multimodal Y,
    Z = a random subset of rank-0 X, perturbed variational state (seeded)."""
    N, M, K, D, ls, S = cfg
    rng = np.random.default_rng(1000 + rank)
    X = rng.standard_normal((N, D)).astype(np.float32)
    w = np.random.default_rng(1).standard_normal((K, D)) / np.sqrt(D)
    c = np.arange(N) % K
    Y = (np.sin(np.sum(w[c] * X, 1) + c) + 0.1 * rng.standard_normal(N)).astype(np.float32)
    X0 = np.random.default_rng(1000).standard_normal((N, D)).astype(np.float32)
    Zf = X0[np.random.default_rng(2).choice(N, M, replace=False)]
    Za = X0[np.random.default_rng(3).choice(N, M, replace=False)]
    r4 = np.random.default_rng(4)
    layers = []
    for Z, var in ((Zf, 0.5), (Za, 0.1)):
        q_mu = (0.5 * r4.standard_normal((M, K))).astype(np.float32)
        q_sqrt = np.empty((K, M, M), np.float32)
        for k in range(K):
            q_sqrt[k] = 0.5 * np.eye(M, dtype=np.float32) + np.tril(
                0.1 * r4.standard_normal((M, M)).astype(np.float32))
        layers.append((Z, var, q_mu, q_sqrt))
    return X, Y, layers


def build_model(cfg, layers, device, num_data):
    from MixtureGPs.likelihoods import GaussianModified
    from MixtureGPs.models import SMGP, SVGPModified
    from modulatedgps_amd.kernels import SquaredExponential
    N, M, K, D, ls, S = cfg
    lik = GaussianModified(variance=0.5, D=K, device=device)
    svgp = []
    for Z, var, q_mu, q_sqrt in layers:
        kern = SquaredExponential(variance=var, lengthscales=ls, device=device)
        layer = SVGPModified(kernel=kern, likelihood=lik, inducing_variable=Z, num_latent_gps=K,
                             whiten=True, device=device)
        layer.set_variational(torch.from_numpy(q_mu), torch.from_numpy(q_sqrt))
        svgp.append(layer)
    return SMGP(likelihood=lik, pred_layer=svgp[0], assign_layer=svgp[1], K=K, num_samples=S,
                num_data=num_data, seed=1234)


def stage_stats(timing):
    """{stage: (avg ms per launch, launches)} from recorded HIP event pairs."""
    out = {}
    for name, pairs in timing.items():
        ts = [a.elapsed_time(b) for a, b in pairs]
        out[name] = (float(np.mean(ts)), len(ts))
    return out


def cpu_baseline(cfg, sizes):
    """Float64 oracle (oracle/cpu_ref.py, S-deduplicated restatement of the reference
    semantics) timed on this host's cores on a bounded sample: config shapes with N
    reduced to `sizes`, t(N) = a + b N fitted and extrapolated to the full N."""
    from oracle import cpu_ref as R
    try:
        from threadpoolctl import threadpool_info
        cores = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        cores = os.cpu_count()
    Nfull, M, K, D, ls, S = cfg
    ts = []
    for n in sizes:
        X, Y, p = R.synthetic_problem(n, M, K, D, ls, state="perturbed", S=S)
        z, u = R.explicit_noise(S, n, K)
        R.smgp_elbo(X[:256], Y[:256], p, z[:, :256], u[:, :256])   # warm BLAS
        t0 = time.perf_counter()
        R.smgp_elbo(X, Y, p, z, u)
        ts.append(time.perf_counter() - t0)
    b = (ts[1] - ts[0]) / (sizes[1] - sizes[0])
    a = max(ts[0] - b * sizes[0], 0.0)
    if Nfull in sizes:
        t_full = ts[list(sizes).index(Nfull)]
        how = f"timed directly at N={Nfull}"
    else:
        t_full = a + b * Nfull
        how = f"t = a + b N extrapolated to N={Nfull}"
    return {"value": 1.0 / t_full, "unit": "ELBO steps/s", "cores": int(cores), "kind": "port",
            "sample": (f"one float64 ELBO of the oracle (oracle/cpu_ref.py; reference semantics, "
                       f"S-deduplicated, TF2 unavailable) at M={M},K={K},D={D},S={S}: N={sizes[0]} "
                       f"took {ts[0]:.2f}s, N={sizes[1]} took {ts[1]:.2f}s; {how}: {t_full:.2f}s per ELBO"),
            "seconds_per_step": t_full}


def probe_kuf(model, X, x6, reps=20, fmt="x6"):
    """K1 launch time without the step's concurrency: `reps` back-to-back launches
    between two HIP events on the current stream (in the step, K1 shares the GPU
    with K3 on a side stream and its event bracket includes host submission)."""
    from modulatedgps_amd import ops
    layer = model.pred_layer
    b = model._buffers(X.shape[0])
    if x6:
        fn = lambda: ops.rbf_kuf_x6(X, layer.Z, layer.kernel.variance, layer.kernel.lengthscales,
                                    out=b["Kfr_f"], fmt=fmt)
    else:
        fn = lambda: ops.rbf_kuf(X, layer.Z, layer.kernel.variance, layer.kernel.lengthscales,
                                 out=b["Kuf_f"])
    fn()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def load_traffic(kernel):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    e = d.get("kernels", d).get(kernel)
    if not e:
        return None, None
    return e.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def k5_modes_leg(elbo_step, args, fmt, steps=10):
    """Side measurement (never the headline): the same ELBO step with the other
    f32-accurate image format, and with K5 on 2 and 1 bf16 planes (BASELINE config
    5's 'bf16 mixed'); their measured fvar error vs the float64 oracle at c3 shapes
    is asserted in tests/test_gpu_kernels.py::test_expert_conditional_planes (2
    planes ~3e-6, 1 plane ~2e-3 normwise) and tests/test_gpu_f16.py."""
    from modulatedgps_amd.config import expert_cross, set_expert_cross, set_expert_format, set_expert_planes
    out = {}
    cross = expert_cross()
    if fmt == "f16":  # the other cross-term precision on the same images
        set_expert_cross("f16" if cross == "f8" else "f8")
        for _ in range(2):
            elbo_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            elbo_step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        out["f16x3" if cross == "f8" else "f16x8"] = {
            "value": 1.0 / dt, "unit": "ELBO steps/s", "ms_per_step": dt * 1e3,
            "k5_f16_product_equivalents": 3 if cross == "f8" else 2,
            "accuracy": ("f32 class (tests/test_gpu_f16.py)" if cross == "f8" else
                         "fvar 6.4e-6 normwise vs float64 at c3 shapes (f32 class: 7e-7; "
                         "tests/test_gpu_f16.py, gate 1e-4)")}
        set_expert_cross(cross)
    other = "x6" if fmt == "f16" else "f16"
    set_expert_format(other)
    for _ in range(2):
        elbo_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        elbo_step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out[other] = {"value": 1.0 / dt, "unit": "ELBO steps/s", "ms_per_step": dt * 1e3,
                  "k5_products": 6 if other == "x6" else 3, "accuracy": "f32 class (tests/test_gpu_f16.py)"}
    set_expert_format("x6")
    for planes in (2, 1):
        set_expert_planes(planes)
        for _ in range(2):
            elbo_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            elbo_step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        out[f"planes{planes}"] = {"value": 1.0 / dt, "unit": "ELBO steps/s", "ms_per_step": dt * 1e3,
                                  "k5_products": planes * (planes + 1) // 2,
                                  "fvar_normwise_err_vs_f64": {2: "3.3e-6", 1: "2.1e-3"}[planes]}
    set_expert_planes(3)
    set_expert_format(fmt)
    return out


def train_leg(model, X, Y, kw, args, barrier, world, device, units):
    """Secondary line: the run_adam optimisation step (utils/training_utils.py:10-13:
    ELBO, its gradient w.r.t. every trainable parameter, one TF-legacy Adam update),
    same workload and timing protocol as the forward leg."""
    from modulatedgps_amd.training import AdamTF
    opt = AdamTF(model.trainable_parameters(), 1e-3)

    from modulatedgps_amd.models import _Stage

    def step(timing=None):
        e, g = model.elbo_and_grad(X, Y, timing=timing, **kw)
        with _Stage(timing, "adam"):
            opt.step(g)
        return e

    for _ in range(max(1, args.warmup)):
        step()
    steps = max(args.repeats, min(args.steps, 50))   # ~1 s of training steps at c3
    blocks, e = timed_blocks(step, steps, args.repeats, barrier, world, device)
    value, ms, rates = median_rate(blocks, units)
    timing = {}   # stage brackets in an untimed block (see main)
    stage_steps = min(10, steps)
    timed_blocks(step, stage_steps, 1, barrier, world, device, timing)
    st = stage_stats(timing)
    return {"metric": "training steps/sec (forward + full gradient + Adam)", "value": value,
            "unit": "train steps/s", "ms_per_step": ms, "steps": steps, "block_rates": rates,
            "elbo_last": float(e.item()),
            "stages_us_per_step": {k: round(v[0] * v[1] / stage_steps * 1e3, 1) for k, v in st.items()}}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args)
    from modulatedgps_amd.config import (conditional_mode, expert_cross, expert_format, set_expert_cross,
                                         set_expert_format, set_expert_planes)
    x6 = conditional_mode() == "x6"
    set_expert_planes(args.planes)
    fmt = args.format or expert_format()
    set_expert_format(fmt)
    set_expert_cross(args.cross or expert_cross())
    f16 = x6 and fmt == "f16" and args.planes == 3
    f16x8 = f16 and expert_cross() == "f8"
    # 6 / 3 / 1 bf16 MFMA products per f32 product; split-f16: 3 f16 products (same rate);
    # f16x8: 1 f16 product + half an e4m3 32x32x64 MFMA (2x rate) = 2 f16-product equivalents
    k5_products = (2 if f16x8 else 3) if f16 else args.planes * (args.planes + 1) // 2
    peak_k5 = PEAK_BF16_MFMA / k5_products if x6 else PEAK_F32_MFMA
    from modulatedgps_amd.distributed import init_from_env
    # MGP_BENCH_BACKEND=gloo + MGP_BENCH_SHARE_GPU=1: rehearsal of the multi-rank path
    # with every rank on cuda:0 (a one-GPU box); the driver's runs use RCCL, one GPU per rank
    share = os.environ.get("MGP_BENCH_SHARE_GPU") == "1"
    if share:
        os.environ["LOCAL_RANK"] = "0"
    rank, world, local = init_from_env(os.environ.get("MGP_BENCH_BACKEND", "nccl"))
    group = torch.distributed.group.WORLD if world > 1 else None
    device = torch.device("cuda", local if world > 1 else 0)
    cfg = CONFIGS[args.config]
    expert = args.layout == "expert" and world > 1
    strong = args.scaling == "strong" and not expert and world > 1
    if strong:  # c4: the config's N split over the ranks (balanced shards)
        from modulatedgps_amd.distributed import shard_rows
        lo, hi = shard_rows(cfg[0], rank, world)
        cfg = (hi - lo,) + tuple(cfg[1:])
    N, M, K, D, ls, S = cfg
    X_np, Y_np, layers = synthetic(cfg, 0 if expert else rank, device)
    if strong:
        n_total, n_offset = CONFIGS[args.config][0], lo
    else:
        n_total, n_offset = (N if expert else N * world), rank * N
    model = build_model(cfg, layers, device, num_data=n_total)
    X = torch.from_numpy(X_np).to(device)
    Y = torch.from_numpy(Y_np).to(device)
    kw = dict(n_offset=n_offset, n_total=n_total, process_group=group)
    if expert:
        from modulatedgps_amd.distributed import expert_parallel_elbo

        def elbo_step(timing=None):
            return expert_parallel_elbo(model, X, Y, group=group)
    else:
        def elbo_step(timing=None):
            return model._build_likelihood(X, Y, timing=timing, **kw)

    for _ in range(args.warmup):
        elbo_step()
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    blocks, elbo = timed_blocks(elbo_step, args.steps, args.repeats, barrier, world, device)
    elbo_val = float(elbo.item())
    info = model.last_info.cpu().tolist() if model.last_info is not None else None
    # per-stage event brackets in a separate, untimed block: an event record between
    # two kernels costs ~10 us of idle GPU, so the timed steps carry none
    timing = {}
    stage_steps = min(20, args.steps)
    timed_blocks(elbo_step, stage_steps, 1, barrier, world, device, timing)
    st = stage_stats(timing)

    # algorithmic work per launch
    if x6:   # K1 writes the split-bf16 image of Kuf (6 B per element of the padded [Mp, Np];
        # split-f16: 4 B)
        Mp, Np = -(-M // 128) * 128, -(-N // 256) * 256
        kuf_bytes = 4.0 * (N * D + M * D) + (4.0 if f16 else 6.0) * Mp * Np
    else:
        kuf_bytes = 4.0 * (N * D + M * D + M * N)
    trsm_flops = float(M) * M * N
    expert_flops = float(K) * M * M * N
    chol_flops = 2 * (2.0 * M ** 3 / 3.0)        # potrf + trtri, both layers (one batched sweep)
    kernels = {}
    from modulatedgps_amd.config import step_schedule
    if "rbf_kuf" in st or (x6 and step_schedule() == "k1_in_k3"):
        ms = probe_kuf(model, X, x6, fmt="f16" if f16 else "x6")
        kernels["rbf_kuf"] = {"bound": "hbm", "avg_us": ms * 1e3, "bytes": kuf_bytes,
                              "achieved": kuf_bytes / (ms * 1e-3) / 1e9, "unit": "GB/s",
                              "peak": PEAK_HBM / 1e9, "frac": kuf_bytes / (ms * 1e-3) / PEAK_HBM,
                              "timing": "20 back-to-back launches after the timed steps (rbf_kuf_x6_kernel)"}
        if "rbf_kuf" in st:
            kernels["rbf_kuf"]["in_step_avg_us"] = st["rbf_kuf"][0] * 1e3
        else:   # the step's K1 is a side job of K3's step launches (mgp_kuu_potrf_trtri_kuf)
            kernels["rbf_kuf"]["in_step"] = "inside kuu_chol: the same image blocks on idle CUs of K3's step launches"
    # both layers' K4 (and K5) run as one launch each in the default schedule: a launch's
    # algorithmic work is then twice one layer's
    lpl = int(getattr(model, "layers_per_launch", 1))
    trsm_flops *= lpl
    expert_flops *= lpl
    for name, fl, peak in (("trsm_stats", trsm_flops, (PEAK_BF16_MFMA / 3 if f16 else PEAK_X6) if x6 else PEAK_F32_MFMA),
                           ("expert_cond", expert_flops, peak_k5)):
        if name in st:
            ms = st[name][0]
            kernels[name] = {"bound": "mfma", "avg_us": ms * 1e3, "flops": fl, "layers_per_launch": lpl,
                             "achieved": fl / (ms * 1e-3) / 1e12, "unit": "TFLOP/s",
                             "peak": peak / 1e12, "frac": fl / (ms * 1e-3) / peak}
    if "kuu_chol" in st:
        ms = st["kuu_chol"][0]
        kernels["kuu_chol"] = {"bound": "latency", "avg_us": ms * 1e3, "flops": chol_flops,
                               "achieved": chol_flops / (ms * 1e-3) / 1e12, "unit": "TFLOP/s",
                               "peak": PEAK_F64 / 1e12, "frac": chol_flops / (ms * 1e-3) / PEAK_F64}
    for name in ("elbo_terms", "gauss_kl", "allreduce", "split_tri"):
        if name in st:
            kernels[name] = {"avg_us": st[name][0] * 1e3}

    ek = kernels.get("expert_cond", {})
    kname = (("expert_cond_f16x8_kernel" if f16x8 else
              ("expert_cond16_pair_kernel" if lpl == 2 else "expert_cond16_kernel")) if f16 else
             "expert_cond_x6_kernel") if x6 else "expert_cond_kernel"
    traffic, traffic_src = load_traffic(kname)
    klabel = {"expert_cond16_kernel": "expert_cond16_kernel<false> (split-f16, 16x16x32 MFMA)",
              "expert_cond16_pair_kernel": "expert_cond16_pair_kernel<false> (split-f16, 16x16x32 MFMA, "
                                           "both layers in one launch)",
              "expert_cond_f16x8_kernel": "expert_cond_x6_kernel<2, true, true> (split-f16 + e4m3 cross terms)"
              }.get(kname, kname)
    roofline = {"kernel": f"{klabel} (K5, L_k^T A + sum of squares, + cond_finalize)", "bound": "mfma",
                "achieved": ek.get("achieved"), "peak": peak_k5 / 1e12,
                "unit": "TFLOP/s", "frac": ek.get("frac"), "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_per_launch": f"{lpl}*K*M^2*N = {expert_flops:.4g} f32 flop" if lpl > 1 else
                                          f"K*M^2*N = {expert_flops:.4g} f32 flop",
                "peak_note": ("split-f16 + e4m3 cross terms: each f32 product is 1 f16 MFMA product + both "
                              "cross products at e4m3 (2x rate), peak = 2.5 PF f16 dense / 2" if f16x8 else
                              "split-f16: each f32 product is 3 f16 MFMA products, peak = 2.5 PF f16 dense / 3"
                              if f16 else
                              f"split-bf16: each f32 product is {k5_products} bf16 MFMA products, peak = "
                              f"2.5 PF bf16 dense / {k5_products}" if x6 else "f32 MFMA dense peak")}

    # ELBO steps/s in units of whole-config evaluations: weak = world evaluations of
    # N points per step; strong / expert = one evaluation of the config's N per step
    units = 1 if (expert or strong) else world
    value, ms_per_step, block_rates = median_rate(blocks, units)
    train = None if (args.no_train or expert) else train_leg(model, X, Y, kw, args, barrier, world, device, units)
    modes = None
    if world == 1 and x6 and args.planes == 3 and not args.no_modes:
        modes = k5_modes_leg(elbo_step, args, fmt)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sizes = tuple(args.cpu_sample)
        if cfg[0] < max(sizes):   # c4r / c2: sample at and below the config's own N
            sizes = (cfg[0] // 4, cfg[0])
        cpu = cpu_baseline(cfg, sizes)
    step_flops = 2 * (2.0 * M ** 3 / 3.0 + (K + 1.0) * M * M * N + N * M * (3 * D + 4.0))
    if rank == 0:
        out = {
            "metric": ("ELBO steps/sec (N=65536, M=1024, K=8); Kuf HBM GB/s vs roofline" if args.config == "c3" else
                       f"ELBO steps/sec (N={CONFIGS[args.config][0]}, M={M}, K={K}); Kuf HBM GB/s vs roofline"),
            "value": value, "unit": "ELBO steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            # N = 1: both layouts are the same run; it is reported under the chosen series
            "scaling": "strong" if (expert or strong or (world == 1 and args.scaling == "strong")) else "weak",
            "vs_baseline": None,
            "repeats": len(blocks), "steps_per_repeat": [n for n, _ in blocks], "block_rates": block_rates,
            "dtype": (("f32 (split-f16 + e4m3 cross terms)" if f16x8 else "f32 (split-f16, 22-bit operands)")
                      if f16 else {3: "f32 (split-bf16 x6, f32-exact operands)", 2: "f32/bf16x3 mixed",
                                   1: "f32/bf16 mixed"}[args.planes]) if x6 else "f32",
            "data": "synthetic",
            "dtype_note": (("f32 operands and accumulation; the forward chain K1 -> K4 -> K5 on f16 MFMA via "
                            "power-of-two-scaled 2-plane fp16 splits (22-bit operands, 3 products), in the ELBO "
                            "and the training step alike; the training backward's g_Lm gram (g_Kuf A^T) and its "
                            "M x M products on bf16 MFMA via an exact 3-plane split (6 products); K3 in f64")
                           + ("; K5's two cross terms (2^-11 of the leading product) on the e4m3 MFMA"
                              if f16x8 else "")
                           if f16 else
                           ("f32 operands and accumulation; K5 products on bf16 MFMA via an exact "
                            "3-plane split (6 products, f32-accurate); K3 in f64") if x6 and args.planes == 3 else
                           (f"K1-K4 f32-accurate (x6 split-bf16), K5 on the leading {args.planes} bf16 plane(s) "
                            f"({k5_products} product(s), f32 accumulation); K3 in f64") if x6 else
                           "f32 MFMA (exact f32); K3 in f64"),
            "config": {"workload": (f"c4 ({args.config} N={n_total} sharded over {world} GPUs): " if strong else
                                     f"{args.config}: ") + f"SMGP ELBO forward, N={N}/GPU, M={M}, K={K}, "
                                    f"D={D}, S={S}, lengthscale={ls}",
                       "global_batch": n_total, "N_per_gpu": N, "M": M, "K": K, "D": D, "S": S,
                       "parallelism": (f"ep{world} (K experts sharded over ranks on N={N}, one RCCL all_to_all of "
                                       f"the conditionals + one scalar all-reduce)" if expert else
                                       f"dp{world} (N-sharded, scalar RCCL all-reduce)")},
            "roofline": roofline,
            "kernels": kernels,
            "kuf_hbm": kernels.get("rbf_kuf"),
            "step_tflops": step_flops / (ms_per_step * 1e-3) / 1e12,
            "step_tflops_note": "f32-equivalent flops of the whole step (both layers) / wall time",
            "cpu_baseline": cpu,
            "train": train,
            "k5_modes": modes,
            "k5_image_format": fmt if x6 else None,
            "k5_cross_terms": expert_cross() if f16 else None,
            "elbo": elbo_val, "cholesky_info": info,
        }
        print(json.dumps(out))
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
