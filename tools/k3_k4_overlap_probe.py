"""Probe: how much does K4 (both layers' triangular solve, trsm_stats16_pair_kernel) slow the
K3 chain when it runs beside it, and how long does it take there?  (Feasibility of
overlapping K4's row tiles with the K3 steps that finalise their L^-1 rows.)

    python tools/k3_k4_overlap_probe.py [reps] [N]

Times, with HIP events, (a) K3 alone (both layers, with the Kuf side job: the ELBO step's
form), (b) the K4 pair alone, (c) K3 on one stream and the K4 pair on a second stream
started once K3's prep is done (K4 on the previous factor's images: timing only).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    M, K, D = 1024, 8, 8
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, D, device=dev, generator=g)
    Z = X[:M].clone()
    var = torch.tensor([0.5], device=dev)
    ls = torch.tensor([1.0], device=dev)
    q_mu = 0.5 * torch.randn(M, K, device=dev, generator=g)
    nb = ops._lib.load().mgp_x6_cols_bytes(M, N)
    K1 = [torch.zeros(nb, dtype=torch.uint8, device=dev) for _ in range(2)]
    _, LinvT, info = ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6, kuf=(X, K1, "f16"))
    Thr = [ops.split_upper_x6(LinvT[b], fmt="f16") for b in range(2)]
    Ahr = [torch.empty_like(K1[0]) for _ in range(2)]
    T = ops.stats_tiles(M)
    sts = [ops.padded(T * (K + 1), N, dev).unflatten(0, (T, K + 1)) for _ in range(2)]
    side = torch.cuda.Stream(device=dev)
    prep = torch.cuda.Event()

    def k3(ev=None):
        ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6, LinvT=LinvT, info=info, kuf=(X, K1, "f16"),
                            prep_event=ev)

    def k4():
        ops.trsm_stats_f16_batch(Thr, K1, [q_mu, q_mu], M, N, Ahr, sts, [var, var])

    def timed(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    for f in (k3, k4):
        f()
    t3 = timed(k3, reps)
    t4 = timed(k4, reps)

    def both():
        k3(prep)
        side.wait_event(prep)
        with torch.cuda.stream(side):
            k4()
        torch.cuda.current_stream().wait_stream(side)

    both()
    tb = timed(both, reps)
    # K3's own span inside the overlapped pair: events on its stream around it
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    spans = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0.record()
        k3(prep)
        e1.record()
        side.wait_event(prep)
        with torch.cuda.stream(side):
            k4()
            e2.record(side)
        torch.cuda.synchronize()
        spans.append((e0.elapsed_time(e1) * 1e3, e0.elapsed_time(e2) * 1e3))
    k3s = sorted(s[0] for s in spans)[len(spans) // 2]
    k4e = sorted(s[1] for s in spans)[len(spans) // 2]
    print(f"K3 alone {t3:.1f} us  K4 pair alone {t4:.1f} us  sum {t3 + t4:.1f} us")
    print(f"overlapped: pair wall {tb:.1f} us; K3 span {k3s:.1f} us, K4 done at {k4e:.1f} us after K3's start")


if __name__ == "__main__":
    main()
