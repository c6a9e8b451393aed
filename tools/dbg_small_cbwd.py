"""Debug: the conditional backward's outputs at tiny N against float64 autograd at
the device's own A (as tests/test_gpu_backward.py::test_conditional_backward)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import cpu_ref as R  # noqa: E402
from tests.helpers import normwise, to_np  # noqa: E402
from modulatedgps_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
f32 = lambda a: np.asarray(a, np.float32)
for (N, M, K, D, ls) in [(2, 1, 1, 1, 0.5), (3, 1, 1, 1, 0.5), (5, 1, 1, 1, 0.5), (8, 1, 1, 1, 0.5), (2, 2, 1, 1, 0.5),
                         (40, 3, 2, 1, 0.5), (300, 20, 3, 2, 0.8)]:
    rng = np.random.default_rng(7)
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=2)
    L = p.pred
    Xt, Zt = torch.as_tensor(f32(X), device=dev), torch.as_tensor(f32(L["Z"]), device=dev)
    var = torch.as_tensor([L["variance"]], dtype=torch.float32, device=dev)
    lst = torch.as_tensor([ls], dtype=torch.float32, device=dev)
    qmu = torch.as_tensor(f32(L["q_mu"]), device=dev)
    qs = ops.as_padded(torch.as_tensor(f32(L["q_sqrt"])), device=dev)
    gmu = rng.standard_normal((K, N)).astype(np.float32)
    gv = rng.standard_normal((K, N)).astype(np.float32)
    Gmu, Gv = ops.padded(K, N, dev), ops.padded(K, N, dev)
    Gmu.copy_(torch.as_tensor(gmu))
    Gv.copy_(torch.as_tensor(gv))
    _, LinvT, _ = ops.kuu_potrf_trtri([Zt], [var], [lst], 1e-6)
    Khr = ops.rbf_kuf_x6(Xt, Zt, var, lst, fmt="f16")
    Thr = ops.split_upper_x6(LinvT[0], fmt="f16")
    A = ops.padded(M, N, dev)
    Ahr, sth = ops.trsm_stats_x6(Thr, Khr, qmu, M, N, A=A, f16_variance=var, in_fmt="f16", cross="f16")
    Lhr = ops.split_lower_x6(qs, fmt="f16")
    Cfr = torch.empty(ops.c_images_bytes(M, N, K), dtype=torch.uint8, device=dev)
    colmax = ops.colnorm_max(qs)
    ops.expert_conditional_x6(Ahr, Lhr, sth, var, M, N, K, fmt="f16", cross="f16", c_out=(Cfr, colmax))
    outs = {"c": ops.conditional_backward_x6(Ahr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N, fmt="f16", cross="f16",
                                             c_images=(Cfr, colmax, ops.image_bound(Lhr, M, K=K))),
            "s": ops.conditional_backward_x6(Ahr, A, qs, qmu, LinvT[0], Gmu, Gv, M, N, fmt="f16", cross="f16")}
    A64 = torch.tensor(to_np(A)[:, :N], requires_grad=True)
    Linv = to_np(LinvT[0]).T
    q_mu = torch.tensor(f32(L["q_mu"]).astype(np.float64), requires_grad=True)
    q_sqrt = torch.tensor(f32(L["q_sqrt"]).astype(np.float64), requires_grad=True)
    v = torch.tensor(float(np.float32(L["variance"])), dtype=torch.float64, requires_grad=True)
    fmean = (A64.T @ q_mu).T
    LTA = torch.tril(q_sqrt).transpose(1, 2) @ A64
    fvar = v - (A64 ** 2).sum(0)[None, :] + (LTA ** 2).sum(1)
    loss = (torch.tensor(gmu.astype(np.float64)) * fmean).sum() + (torch.tensor(gv.astype(np.float64)) * fvar).sum()
    loss.backward()
    gKuf_ref = Linv.T @ A64.grad.numpy()
    gLm_ref = -np.tril(gKuf_ref @ A64.detach().numpy().T)
    for tag, g in outs.items():
        e = {"g_Kuf": normwise(to_np(g["g_Kuf"])[:, :N], gKuf_ref), "g_Lm": normwise(to_np(g["g_Lm"]), gLm_ref),
             "g_q_mu": normwise(to_np(g["g_q_mu"]), q_mu.grad.numpy()),
             "g_q_sqrt": normwise(to_np(g["g_q_sqrt"]), np.tril(q_sqrt.grad.numpy())),
             "g_var": abs(float(g["g_var"].cpu()) - float(v.grad)) / abs(float(v.grad))}
        print((N, M, K, D), tag, {k: f"{x:.1e}" for k, x in e.items()}, flush=True)
        if max(e.values()) > 1e-3:
            print("   q_sqrt got", to_np(g["g_q_sqrt"]).ravel()[:4], "ref", np.tril(q_sqrt.grad.numpy()).ravel()[:4])
            print("   g_Kuf got", to_np(g["g_Kuf"])[:, :N].ravel()[:4], "ref", gKuf_ref.ravel()[:4])
            print("   g_var got", float(g["g_var"].cpu()), "ref", float(v.grad), "A", to_np(A)[:, :N].ravel()[:4])
