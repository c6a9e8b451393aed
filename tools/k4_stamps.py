"""K4 (trsm_stats16_kernel) phase times per workgroup from in-kernel stamps on the
100 MHz reference clock (GPU box only).  Rebuilds libmgp_hip.so with
-DMGP_DBG_STAMPS in this (scratch) tree, runs K4 at c3 (M = 1024, N = 65536,
K = 8) and prints: workgroup start times (dispatch rounds), per item the main
loop (from the item's start, so its prologue is included) against its k-step
pairs, and the epilogues.
Usage: python tools/k4_stamps.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import build as B  # noqa: E402

B.build(extra_flags=["-DMGP_DBG_STAMPS"])
import torch  # noqa: E402
from modulatedgps_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda", 0)
M, N, K, D = 1024, 65536, 8, 8
g = torch.Generator(device=dev).manual_seed(0)
Z = torch.randn(M, D, device=dev, generator=g)
X = torch.randn(N, D, device=dev, generator=g)
var = torch.tensor([0.5], device=dev)
ls = torch.tensor([1.0], device=dev)
q_mu = ops.as_padded(torch.randn(M, K, device=dev, generator=g) * 0.1, dev)
_, LinvT, _ = ops.kuu_potrf_trtri([Z], [var], [ls], 1e-6)
Khr = ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16")
Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
Ahr = torch.empty(_lib.load().mgp_x6_cols_bytes(M, N), dtype=torch.uint8, device=dev)
nT = M // 128
st = None
for _ in range(5):
    _, st = ops.trsm_stats_x6(Thr, Khr, q_mu, M, N, Afr=Ahr, stats=st, f16_variance=var, in_fmt="f16", cross="f16")
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (4096 * 8))()
_lib.load().mgp_dbg_k4_stamps(buf)
nP, nTn = (nT + 1) // 2, N // 256
nwg = nP * nTn
s = np.array([[buf[b * 8 + k] for k in range(5)] for b in range(nwg)], dtype=np.float64)
t0 = s[:, 0].min()
s = (s - t0) * 0.01  # us
b = np.arange(nwg)
j = b >> 3
p = nP - 1 - j % nP
t1, t2 = nT - 1 - p, p
pairs1, pairs2 = 4 * (t1 + 1), 4 * (t2 + 1)
print(f"K4 at c3: {nwg} row-tile-pair items; kernel span {s[:, 4].max():.1f} us")
starts = np.sort(s[:, 0])
print("item start times (us): percentiles 0/25/50/75/100:",
      " ".join(f"{np.percentile(starts, q):.1f}" for q in (0, 25, 50, 75, 100)))
print("  started within 5 us of the first:", int((starts < 5).sum()), " after 50 us:", int((starts > 50).sum()))
loop1, epi1 = s[:, 1] - s[:, 0], s[:, 2] - s[:, 1]
loop2, epi2 = s[:, 3] - s[:, 2], s[:, 4] - s[:, 3]
print("item   pairs  workgroups  loop+prologue us (median)  per pair us  epilogue us (median)")
for pp in range(nP):
    m = p == pp
    for name, pr, lp, ep in (("first", pairs1, loop1, epi1), ("second", pairs2, loop2, epi2)):
        npairs = int(pr[m][0])
        print(f"{name:6s} {npairs:5d}  {int(m.sum()):10d}  {np.median(lp[m]):24.2f}  {np.median(lp[m]) / npairs:11.3f}"
              f"  {np.median(ep[m]):8.2f}")
# least squares: loop = a + c * pairs over both items of every workgroup
x = np.concatenate([pairs1, pairs2]).astype(np.float64)
y = np.concatenate([loop1, loop2])
A = np.stack([np.ones_like(x), x], 1)
(a, c), *_ = np.linalg.lstsq(A, y, rcond=None)
print(f"fit: item main loop = {a:.2f} us + {c:.3f} us per k-step pair  (prologue / fixed cost per item {a:.2f} us)")
print(f"epilogue median {np.median(np.concatenate([epi1, epi2])):.2f} us;"
      f" workgroup busy median {np.median(s[:, 4] - s[:, 0]):.1f} us")
busy = s[:, 4] - s[:, 0]
print("workgroup busy us percentiles 0/10/50/90/100:", " ".join(f"{np.percentile(busy, q):.1f}" for q in (0, 10, 50, 90, 100)))
r1 = s[:, 0] < 5
print(f"round 1: {int(r1.sum())} workgroups, end percentiles 0/50/100:",
      " ".join(f"{np.percentile(s[r1, 4], q):.1f}" for q in (0, 50, 100)),
      f"| round 2: {int((~r1).sum())}, busy median {np.median(busy[~r1]):.1f} us")
for x in range(8):
    m = (b % 8) == x
    print(f"  XCD {x} (block % 8): busy median {np.median(busy[m]):.1f} us, round-1 end median "
          f"{np.median(s[m & r1, 4]):.1f} us")
