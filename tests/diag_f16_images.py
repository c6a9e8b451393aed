"""Component accuracy of the split-f16 forward chain (diagnostic, not collected by pytest).

    python -m tests.diag_f16_images [--N 65536 --M 1024 --D 8 --ls 1.0 --vars 0.1,0.5]

Test infrastructure (float64 numpy references).  Per kernel variance: the Kuf image
of K1 (split-f16 and x6) decoded against float64 Kuf, and K4's float32 A (from
split-f16 and from x6 images) against float64 L^-1 Kuf (models.py:139-143).  This is
the probe that found the round-6 K1 split bug (tests/test_gpu_f16.py).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import cpu_ref as R          # noqa: E402
from tests.helpers import decode_cols_f16, normwise, to_np   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--D", type=int, default=8)
    ap.add_argument("--ls", type=float, default=1.0)
    ap.add_argument("--vars", default="0.1,0.5")
    a = ap.parse_args()
    from modulatedgps_amd import ops
    from tests.helpers import decode_cols_image
    dev = torch.device("cuda", 0)
    X, _, p = R.synthetic_problem(a.N, a.M, 1, a.D, a.ls, state="perturbed", S=1)
    Z = p.assign["Z"]
    X32, Z32 = X.astype(np.float32), Z.astype(np.float32)
    Xd, Zd = torch.as_tensor(X32, device=dev), torch.as_tensor(Z32, device=dev)
    ls = torch.tensor([a.ls], dtype=torch.float32, device=dev)
    q_mu = torch.zeros(a.M, 1, dtype=torch.float32, device=dev)
    for v in (float(x) for x in a.vars.split(",")):
        var = torch.tensor([v], dtype=torch.float32, device=dev)
        v32 = float(np.float32(v))
        Kuf64 = R.rbf_K(Z32.astype(np.float64), X32.astype(np.float64), v32, np.float32(a.ls))
        Kuu64 = R.rbf_Kuu(Z32.astype(np.float64), v32, np.float32(a.ls))
        L64 = np.linalg.cholesky(Kuu64)
        A64 = np.linalg.solve(L64, Kuf64)
        rep = {}
        img16 = ops.rbf_kuf_x6(Xd, Zd, var, ls, fmt="f16")
        img6 = ops.rbf_kuf_x6(Xd, Zd, var, ls, fmt="x6")
        kb = float(ops.image_bound(img16, a.M, N=a.N).cpu())
        K16 = decode_cols_f16(img16, a.M, a.N, kb)
        K6 = decode_cols_image(img6, a.M, a.N)
        rep["kuf_bound"] = kb
        rep["kuf_f16"] = normwise(K16, Kuf64)
        rep["kuf_x6"] = normwise(K6, Kuf64)
        rep["kuf_f16_vs_x6_max"] = float(np.abs(K16 - K6).max() / np.abs(K6).max())
        rep["kuf_f16_max_rel_vs_x6"] = float(np.max(np.abs(K16 - K6) / np.maximum(np.abs(K6), 1e-30)))
        LinvT = ops.kuu_potrf_trtri([Zd], [var], [ls], 1e-6)[1][0]
        for fmt, img in (("f16", img16), ("x6", img6)):
            Tfr = ops.split_upper_x6(LinvT, fmt=fmt)
            Af = torch.zeros(a.M, a.N, dtype=torch.float32, device=dev)
            ops.trsm_stats_x6(Tfr, img, q_mu, a.M, a.N, A=Af, f16_variance=var if fmt == "f16" else None,
                              in_fmt=fmt)
            torch.cuda.synchronize()
            Ag = to_np(Af)
            rep["A_" + fmt] = normwise(Ag, A64)
            rep["A_" + fmt + "_maxabs_over_max"] = float(np.abs(Ag - A64).max() / np.abs(A64).max())
            idx = np.unravel_index(np.argmax(np.abs(Ag - A64)), A64.shape)
            rep["A_" + fmt + "_argmax"] = [int(i) for i in idx]
        print(v, json.dumps({k: (f"{x:.3e}" if isinstance(x, float) else x) for k, x in rep.items()}), flush=True)


if __name__ == "__main__":
    main()
