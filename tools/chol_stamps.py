"""K3 critical-path breakdown from in-kernel s_memtime stamps (GPU box only).
Rebuilds libmgp_hip.so with -DMGP_DBG_STAMPS in this (scratch) tree, runs one
batched Kuu Cholesky + inverse at M = 1024, batch 2, and prints per-step
deltas (s_memtime ticks, 100 MHz) of the look-ahead workgroup:
  0 start, 1 tiles loaded, 2 P_i stored, 3 update done, 4 staged, 5 panels
  factored, 6 inverse done, 7 diag written.
--elbo: the stamps of K3 inside bench.py's c3 ELBO step (20 evaluations back to back,
the last one's K3: it follows the previous evaluation's K5, with the step's side work
and the K1 side job as in the bench)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from modulatedgps_amd import build as B  # noqa: E402

B.build(extra_flags=["-DMGP_DBG_STAMPS"])
import torch  # noqa: E402
from modulatedgps_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda", 0)
M = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1024
g = torch.Generator(device=dev).manual_seed(0)
Z = torch.randn(M, 8, device=dev, generator=g)
var = torch.tensor([0.5], device=dev)
ls = torch.tensor([1.0], device=dev)
with_k1 = "--with-k1" in sys.argv   # K1 x 2 on a side stream from the prep on, as in the step
if with_k1:
    N = 65536
    X = torch.randn(N, 8, device=dev, generator=g)
    side = torch.cuda.Stream(device=dev)
    ev = torch.cuda.Event()
    ev.record()
    kfr = [ops.rbf_kuf_x6(X, Z, var, ls, fmt="f16") for _ in range(2)]
elbo = "--elbo" in sys.argv
if elbo:
    import bench
    cfg = bench.CONFIGS["c3"]
    M = cfg[1]
    Xn, Yn, layers = bench.synthetic(cfg, 0, dev)
    model = bench.build_model(cfg, layers, dev, num_data=cfg[0])
    Xe, Ye = torch.from_numpy(Xn).to(dev), torch.from_numpy(Yn).to(dev)
    for _ in range(20):
        model._build_likelihood(Xe, Ye, n_offset=0, n_total=cfg[0], process_group=None)
for _ in range(0 if elbo else 3):
    if with_k1:
        torch.cuda.synchronize()
        ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6, prep_event=ev)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            for k in kfr:
                ops.rbf_kuf_x6(X, Z, var, ls, out=k, fmt="f16")
    else:
        ops.kuu_potrf_trtri([Z, Z], [var, var], [ls, ls], 1e-6)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * (64 * 16))()
lib.mgp_dbg_chol_stamps(buf)
st = [[buf[j * 16 + k] for k in range(16)] for j in range(64)]
steps = M // 64 - 1
print("step  load  P_i  update  stage  panels  inverse  write  | next-step gap  || panel0 upd0 panel1 upd1 panel2 upd2+panel3 | inv-a inv-b")
for j in range(steps):
    s = st[j]
    d = [s[k + 1] - s[k] if s[k + 1] and s[k] else 0 for k in range(7)]
    gap = (st[j + 1][0] - s[7]) if j + 1 < steps and st[j + 1][0] else 0
    sub = [s[8] - s[4], s[9] - s[8], s[10] - s[9], s[11] - s[10], s[12] - s[11], s[5] - s[12], "|",
           s[13] - s[5], s[6] - s[13]] if s[8] else []
    print(j, d[0], d[1], d[2], d[3], s[5] - s[4], s[6] - s[5], s[7] - s[6], "|", gap, "||", *sub)
print("reference clock (100 MHz, one time base): step wall us, shader clock GHz, gap to the next step's look-ahead start us")
for j in range(steps):
    s, n = st[j], st[j + 1] if j + 1 < steps else None
    wall = (s[15] - s[14]) * 1e-2
    clk = (s[7] - s[0]) / max(1, s[15] - s[14]) / 10.0
    gap = (n[14] - s[15]) * 1e-2 if n and n[14] else float("nan")
    print(f"{j:2d} wall {wall:6.2f} us  clock {clk:5.2f} GHz  gap {gap:6.2f} us")
# row preparation (batch entry 0), us after the step's look-ahead start: prep kind 0 start,
# prep kinds 0 / 1 published, the row finish saw both flags (and the S2 phase's start: stamp 11)
rf = (ctypes.c_ulonglong * (64 * 4))()
if hasattr(lib, "mgp_dbg_rf_stamps"):
    lib.mgp_dbg_rf_stamps(rf)
    print("row preparation (us after the look-ahead's start): prep start, kind 0 done, kind 1 done, finish saw flags")
    for j in range(steps):
        t0 = st[j][14]
        v = [rf[j * 4 + k] for k in range(4)]
        if t0 and v[1]:
            print(f"{j:2d} prep {(v[3] - t0) * 1e-2:6.2f}  W' {(v[1] - t0) * 1e-2:6.2f}  F {(v[2] - t0) * 1e-2:6.2f}"
                  f"  seen {(v[0] - t0) * 1e-2 if v[0] else float('nan'):6.2f}")
# one pair workgroup per step (first pair of the last tile row, batch 0): shader cycles per phase
pb = (ctypes.c_ulonglong * (64 * 8))()
lib.mgp_dbg_pair_stamps(pb)
print("pair workgroup (row nb-1, pair 0): loads+stage  P_i+first  stage2  final  store  | total (shader cycles)")
for j in range(steps - 1):
    s = [pb[j * 8 + k] for k in range(8)]
    if not s[0] or not s[5]:
        continue
    d = [s[k + 1] - s[k] for k in range(5)]
    print(j, *d, "|", s[5] - s[0], "| entry->start", s[0] - s[7], " start->loads issued", s[6] - s[0])
# MFMA busy per role (round 6): the analytic f64 MFMA count of the
# workgroup (tools/k3_mfma_count.py: 64 pipe cycles per v_mfma_f64_16x16x4) over its own
# stamped shader cycles on the CU's 4 SIMDs -- the look-ahead workgroup (the factorisation
# chain, VALU panel sweeps) apart from the pair workgroups (the trailing-update / forward-
# substitution GEMMs, north_star's "panel GEMMs")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import k3_mfma_count as KC  # noqa: E402
nb = M // 64
print("MFMA busy per role (analytic MFMAs x 64 cycles / (4 SIMDs x stamped cycles)):")
print("step  look-ahead(cyc, busy)  pair row nb-1 #0 (cyc, MFMAs, busy)")
la_b, pr_b = [], []
for j in range(steps - 1):
    s = st[j]
    la_cyc = s[7] - s[0]
    q = [pb[j * 8 + k] for k in range(8)]
    i, nt, nupd = nb - 1, nb, (nb - 1) - j
    pm = KC.PAIR_P + sum((KC.DIAG if j + 1 + e == i else KC.UPD) if e < nupd else
                         (KC.FWD if e - nupd < j else KC.FWD_DIAG) for e in range(min(2, nt)))
    pc = q[5] - q[0] if q[0] and q[5] else 0
    lb = KC.LOOKAHEAD * 64 / (4 * la_cyc) if la_cyc > 0 else float("nan")
    pbz = pm * 64 / (4 * pc) if pc > 0 else float("nan")
    la_b.append((KC.LOOKAHEAD * 64, 4 * la_cyc))
    if pc:
        pr_b.append((pm * 64, 4 * pc))
    print(f"{j:2d}  {la_cyc:7d} {lb:6.3f}   {pc:7d} {pm:5d} {pbz:6.3f}")
tot = lambda v: sum(a for a, _ in v) / max(1, sum(b for _, b in v))
print(f"cycle-weighted: look-ahead {tot(la_b):.3f}  pair workgroups {tot(pr_b):.3f}")
p = st[63]
if p[0]:
    print(f"prep tile (0, 0): build {p[1] - p[0]}  factor {p[2] - p[1]}  write {p[3] - p[2]} shader cycles; "
          f"wall {(p[15] - p[14]) * 1e-2:.2f} us; first step's look-ahead starts {(st[0][14] - p[15]) * 1e-2:.2f} us later")
