"""Per-stage accuracy of the training gradient (diagnostic, not collected by pytest).

    python -m tests.diag_grad_stages [--N 65536 --M 1024 --K 8 --D 8 --ls 1.0 --S 25]
                                     [--formats f16,x6] [--out FILE.json]

Test infrastructure (it imports oracle/ as the checker, like tests/test_gpu_training.py).
For the problem of test_elbo_and_grad_c3_full it reports, normwise against float64
autograd of oracle/grad_ref.py (the reference graph, models.py:55-79):

  * float32 autograd of the same graph (the bar of the training-gradient test);
  * the HIP gradient per parameter block, per image format;
  * the same with the K6 backward's G = d ELBO / d(fmean, fvar) of both layers replaced
    by the oracle's (so the remaining error is the conditional / Cholesky / RBF backward);
  * the K6 backward's G itself against the oracle's;
  * each layer's conditional-backward outputs (g_Kuf, g_Lm, g_q_mu, g_q_sqrt) given the
    oracle's G, against float64 (and float32) autograd of the layer's conditional.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import cpu_ref as R          # noqa: E402
from oracle import grad_ref as GR        # noqa: E402
from tests.helpers import build_model, dev_noise, normwise, to_np   # noqa: E402


def oracle_grads(X, Y, p, z, u, dtype):
    pred, assign, lik = GR.params_from_oracle(p)
    leaf = lambda t: t.detach().to(dtype).requires_grad_(True)
    pred = {k: leaf(v) for k, v in pred.items()}
    assign = {k: leaf(v) for k, v in assign.items()}
    lik = leaf(lik)
    f = lambda a: torch.tensor(np.asarray(a, np.float32)).to(dtype)
    keep = {}
    e = GR.elbo(f(X), f(Y), pred, assign, lik, f(z), f(u), p.num_data, keep=keep)
    e.backward()
    g = {"lik_variance": lik.grad.double().numpy()}
    for name, L in (("pred", pred), ("assign", assign)):
        for k in GR.LAYER_KEYS:
            gk = L[k].grad.double().numpy()
            g[name + "." + k] = np.tril(gk) if k == "q_sqrt" else gk
    G = {k: keep[k].grad.double().numpy().T.copy() for k in ("mu_f", "var_f", "mu_a", "var_a")}   # [K, N]
    G["_values"] = {k: keep[k].detach().double().numpy().T.copy() for k in ("mu_f", "var_f", "mu_a", "var_a")}
    return float(e.detach()), g, G


def layer_stage_grads(X, L, Gmu, Gv, dtype):
    """Autograd of one layer's conditional (grad_ref.layer_conditional with Kuf and Lm
    kept) for the cotangents (Gmu, Gv) [K, N]: g_Kuf, tril(g_Lm), g_q_mu, tril(g_q_sqrt)."""
    t = lambda a: torch.tensor(np.asarray(a, np.float64)).to(dtype)
    P = {k: t(np.asarray(v, np.float64).astype(np.float32)).requires_grad_(True) for k, v in L.items()}
    Z = P["Z"]
    M = Z.shape[0]
    Kuu = GR.rbf(Z, Z, P["variance"], P["lengthscales"]) + GR.JITTER * torch.eye(M, dtype=dtype)
    Kuu.retain_grad()
    Lm = torch.linalg.cholesky(Kuu)
    Lm.retain_grad()
    Kuf = GR.rbf(Z, t(np.asarray(X, np.float32)), P["variance"], P["lengthscales"])
    Kuf.retain_grad()
    A = torch.linalg.solve_triangular(Lm, Kuf, upper=False)
    fmean = A.T @ P["q_mu"]
    Lk = torch.tril(P["q_sqrt"])
    LTA = Lk.transpose(1, 2) @ A
    fvar = P["variance"] - (A ** 2).sum(0)[:, None] + (LTA ** 2).sum(1).T
    torch.autograd.backward([fmean, fvar], [t(Gmu.T), t(Gv.T)])
    out = {"g_Kuf": Kuf.grad.double().numpy(), "g_Lm": np.tril(Lm.grad.double().numpy()),
           "g_q_mu": P["q_mu"].grad.double().numpy(), "g_q_sqrt": np.tril(P["q_sqrt"].grad.double().numpy())}
    gK = Kuu.grad.double().numpy()
    out["_tail"] = {"g_Kuu": 0.5 * (gK + gK.T)}
    if dtype == torch.float64:   # the tail references (not compared as stages)
        tail = tail_f64(X, L, gKuf=out["g_Kuf"], gKuu=out["_tail"]["g_Kuu"])
        kuf_only = tail_f64(X, L, gKuf=out["g_Kuf"], gKuu=np.zeros_like(gK))
        out["_tail"].update({"g_ls": tail["g_ls"], "g_var_rbf": tail["g_var"], "g_ls_kuf": kuf_only["g_ls"]})
    return out


def tail_f64(X, L, gKuf=None, gKuu=None, gLm=None):
    """float64 autograd of one layer's Kuu / Kuf build and Cholesky from float32
    parameters: with gLm the Cholesky backward (-> gKuu); with gKuf, gKuu the RBF
    backward (-> gZ, g_var, g_ls)."""
    t = lambda a: torch.tensor(np.asarray(a, np.float64))
    P = {k: t(np.asarray(v, np.float64).astype(np.float32)).requires_grad_(True) for k, v in L.items()}
    Z = P["Z"]
    M = Z.shape[0]
    Kuu = GR.rbf(Z, Z, P["variance"], P["lengthscales"]) + GR.JITTER * torch.eye(M, dtype=torch.float64)
    if gLm is not None:
        Kuu_l = Kuu.detach().requires_grad_(True)
        Lm = torch.linalg.cholesky(Kuu_l)
        Lm.backward(t(np.tril(gLm)))
        g = Kuu_l.grad.numpy()
        return 0.5 * (g + g.T)
    Kuf = GR.rbf(Z, t(np.asarray(X, np.float32)), P["variance"], P["lengthscales"])
    ((Kuf * t(gKuf)).sum() + (Kuu * t(gKuu)).sum()).backward()
    return {"gZ": P["Z"].grad.numpy(), "g_var": np.atleast_1d(P["variance"].grad.numpy()),
            "g_ls": np.atleast_1d(P["lengthscales"].grad.numpy())}


def hip_grads(model, X, Y, z, u, device, G_sub=None, capture=None):
    """elbo_and_grad; G_sub: dict of [K, N] arrays written over the K6 backward's G;
    capture: list receiving each conditional backward's outputs (host float64)."""
    from modulatedgps_amd import models, ops
    orig_k6, orig_cb = ops.elbo_terms_backward, ops.conditional_backward_x6
    orig_ch, orig_rb = ops.chol_backward_batch, ops.rbf_backward_batch

    def ch(Ls, LinvTs, gLs, *a, **kw):
        outs = orig_ch(Ls, LinvTs, gLs, *a, **kw)
        if capture is not None:
            capture.append({"chol_in": [to_np(g) for g in gLs], "chol_out": [to_np(o) for o in outs]})
        return outs

    def rb(X, Zs, variances, lengthscales, gKufs, gKuus, gZs, g_vars, g_lss, *a, **kw):
        before = [to_np(g) for g in g_vars]
        out = orig_rb(X, Zs, variances, lengthscales, gKufs, gKuus, gZs, g_vars, g_lss, *a, **kw)
        if capture is not None:
            capture.append({"rbf_gKuf": [to_np(g) for g in gKufs], "rbf_gKuu": [to_np(g) for g in gKuus],
                            "rbf_gZ": [to_np(g) for g in gZs], "rbf_gvar": [to_np(g) - b for g, b in zip(g_vars, before)],
                            "rbf_gls": [to_np(g) for g in g_lss]})
        return out

    def k6(*a, **kw):
        G, glv, glva = orig_k6(*a, **kw)
        if G_sub is not None:
            for i, k in enumerate(("mu_f", "var_f", "mu_a", "var_a")):
                G[i].copy_(torch.as_tensor(G_sub[k], dtype=torch.float32, device=device))
        if capture is not None:
            capture.append({"G": [to_np(G[i]) for i in range(4)]})
        return G, glv, glva

    def cb(*a, **kw):
        out = orig_cb(*a, **kw)
        if capture is not None:
            M = a[7]
            capture.append({k: (np.tril(to_np(v)) if k in ("g_Lm",) else to_np(v)) for k, v in out.items()
                            if k != "g_var"})
            if "g_q_sqrt" in capture[-1]:
                capture[-1]["g_q_sqrt"] = np.tril(capture[-1]["g_q_sqrt"][:, :M, :M])
        return out

    models.ops.elbo_terms_backward, models.ops.conditional_backward_x6 = k6, cb
    models.ops.chol_backward_batch, models.ops.rbf_backward_batch = ch, rb
    try:
        Xd = torch.as_tensor(X, dtype=torch.float32, device=device)
        e, grads = model.elbo_and_grad(Xd, Y, noise=dev_noise(z, u, device))
        torch.cuda.synchronize()
    finally:
        models.ops.elbo_terms_backward, models.ops.conditional_backward_x6 = orig_k6, orig_cb
        models.ops.chol_backward_batch, models.ops.rbf_backward_batch = orig_ch, orig_rb
    return float(e.cpu()), {k: to_np(v) for k, v in grads.items()}


def block_errs(grads, g_ref):
    out = {}
    for n, ref in g_ref.items():
        got = grads[n].reshape(-1) if n.endswith(("variance", "lengthscales")) else grads[n]
        out[n] = normwise(got, ref.reshape(got.shape))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--D", type=int, default=8)
    ap.add_argument("--ls", type=float, default=1.0)
    ap.add_argument("--S", type=int, default=25)
    ap.add_argument("--formats", default="f16,x6")
    ap.add_argument("--stages", action="store_true", help="also the per-layer conditional-backward stages")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from modulatedgps_amd import config
    device = torch.device("cuda", 0)
    t0 = time.time()
    X, Y, p = R.synthetic_problem(a.N, a.M, a.K, a.D, a.ls, state="perturbed", S=a.S)
    z, u = R.explicit_noise(a.S, a.N, a.K, seed=5)
    e64, g64, G64 = oracle_grads(X, Y, p, z, u, torch.float64)
    print(f"oracle f64 {time.time() - t0:.0f}s", flush=True)
    _, g32, G32 = oracle_grads(X, Y, p, z, u, torch.float32)
    V64, V32 = G64.pop("_values"), G32.pop("_values")
    print(f"oracle {time.time() - t0:.0f}s", flush=True)
    rep = {"problem": vars(a), "elbo_f64": e64, "f32_autograd": block_errs(g32, g64),
           "f32_autograd_G": {k: normwise(G32[k], G64[k]) for k in G64},
           "f32_conditionals": {k: normwise(V32[k], V64[k]) for k in V64},
           "f32_conditionals_Gweighted": {k: normwise(V32[k] * G64[k], V64[k] * G64[k]) for k in V64}}
    if a.stages:
        rep["stages_f32_autograd"] = {}
        rep["_stage_ref"] = {}
        for name, L, (gm, gv) in (("pred", p.pred, ("mu_f", "var_f")), ("assign", p.assign, ("mu_a", "var_a"))):
            s64 = layer_stage_grads(X, L, G64[gm], G64[gv], torch.float64)
            s32 = layer_stage_grads(X, L, G64[gm], G64[gv], torch.float32)
            tail = s64.pop("_tail")
            t32 = s32.pop("_tail")
            rep["stages_f32_autograd"][name] = {k: normwise(s32[k], s64[k]) for k in s64}
            # which float32 cotangent moves the lengthscale gradient (float64 tail on each mix)
            rep["stages_f32_autograd"][name]["gKuu"] = normwise(t32["g_Kuu"], tail["g_Kuu"])
            for lab, gf, gu in (("gls_f32Kuf_f32Kuu", s32["g_Kuf"], t32["g_Kuu"]),
                                ("gls_f32Kuf_refKuu", s32["g_Kuf"], tail["g_Kuu"]),
                                ("gls_refKuf_f32Kuu", s64["g_Kuf"], t32["g_Kuu"])):
                rep["stages_f32_autograd"][name][lab] = normwise(tail_f64(X, L, gKuf=gf, gKuu=gu)["g_ls"], tail["g_ls"])
            s64.update(tail)
            rep["_stage_ref"][name] = s64
            print(f"stage oracle {name} {time.time() - t0:.0f}s", flush=True)
        print(f"stage oracle {time.time() - t0:.0f}s", flush=True)
    old = config.expert_format()
    for fmt in a.formats.split(","):
        config.set_expert_format(fmt)
        try:
            model = build_model(p, device)
            cap = []
            e, g = hip_grads(model, X, Y, z, u, device, capture=cap)
            r = {"elbo_rel": abs(e - e64) / abs(e64), "blocks": block_errs(g, g64),
                 "G": {k: normwise(cap[0]["G"][i][:, :a.N], G64[k])
                       for i, k in enumerate(("mu_f", "var_f", "mu_a", "var_a"))}}
            for train in (False, True):
                cond = [to_np(t)[:, :a.N] for t in model.conditionals(
                    torch.as_tensor(X, dtype=torch.float32, device=device), train=train)]
                names = ("mu_f", "var_f", "mu_a", "var_a")
                r["conditionals" + ("_train" if train else "")] = {
                    k: normwise(c, V64[k]) for k, c in zip(names, cond)}
                r["conditionals_Gweighted" + ("_train" if train else "")] = {
                    k: normwise(c * G64[k], V64[k] * G64[k]) for k, c in zip(names, cond)}
            model = build_model(p, device)
            cap = []
            _, g = hip_grads(model, X, Y, z, u, device, G_sub=G64, capture=cap)
            r["blocks_oracle_G"] = block_errs(g, g64)
            if a.stages:
                r["stages_oracle_G"] = {}
                for name, c in zip(("pred", "assign"), cap[1:3]):
                    ref = rep["_stage_ref"][name]
                    M, N = a.M, a.N
                    got = {"g_Kuf": c["g_Kuf"][:M, :N], "g_Lm": c["g_Lm"][:M, :M], "g_q_mu": c["g_q_mu"][:M, :a.K],
                           "g_q_sqrt": c["g_q_sqrt"]}
                    r["stages_oracle_G"][name] = {k: normwise(got[k], ref[k]) for k in got}
                chol = next(c for c in cap if "chol_in" in c)
                rbf = next(c for c in cap if "rbf_gKuf" in c)
                r["tail_oracle_G"] = {}
                for i, (name, L) in enumerate((("pred", p.pred), ("assign", p.assign))):
                    M, N = a.M, a.N
                    gLm = chol["chol_in"][i][:M, :M]
                    gKuu_hip = chol["chol_out"][i][:M, :M]
                    gKuu_f64 = tail_f64(X, L, gLm=gLm)
                    gKuu_ref = rep["_stage_ref"][name]["g_Kuu"]
                    tail = tail_f64(X, L, gKuf=rbf["rbf_gKuf"][i][:M, :N], gKuu=rbf["rbf_gKuu"][i][:M, :M])
                    r["tail_oracle_G"][name] = {
                        "chol_bwd_own": normwise(gKuu_hip, gKuu_f64), "gKuu_vs_oracle": normwise(gKuu_hip, gKuu_ref),
                        "rbf_gZ_own": normwise(rbf["rbf_gZ"][i][:M], tail["gZ"]),
                        "rbf_gls_own": normwise(rbf["rbf_gls"][i].reshape(-1), tail["g_ls"]),
                        "rbf_gvar_own": normwise(rbf["rbf_gvar"][i].reshape(-1), tail["g_var"]),
                        "rbf_gls_ref": normwise(tail["g_ls"], rep["_stage_ref"][name]["g_ls"]),
                        "rbf_gvar_ref": normwise(tail["g_var"], rep["_stage_ref"][name]["g_var_rbf"]),
                        "gls_hipKuf_refKuu": normwise(tail_f64(X, L, gKuf=rbf["rbf_gKuf"][i][:M, :N],
                                                               gKuu=gKuu_ref)["g_ls"],
                                                      rep["_stage_ref"][name]["g_ls"]),
                        "gls_refKuf_hipKuu": normwise(tail_f64(X, L, gKuf=rep["_stage_ref"][name]["g_Kuf"],
                                                               gKuu=rbf["rbf_gKuu"][i][:M, :M])["g_ls"],
                                                      rep["_stage_ref"][name]["g_ls"]),
                        "gls_kuf_part_over_total": float(np.abs(rep["_stage_ref"][name]["g_ls_kuf"]).sum()
                                                         / max(np.abs(rep["_stage_ref"][name]["g_ls"]).sum(), 1e-300))}
        finally:
            config.set_expert_format(old)
        rep[fmt] = r
        print(fmt, json.dumps({k: ({kk: f"{vv:.2e}" for kk, vv in v.items()} if isinstance(v, dict) else v)
                               for k, v in r.items() if k not in ("stages_oracle_G", "tail_oracle_G")}), flush=True)
        if a.stages:
            for key in ("stages_oracle_G", "tail_oracle_G"):
                print(fmt, key, json.dumps({L: {k: f"{v:.2e}" for k, v in d.items()}
                                            for L, d in r[key].items()}), flush=True)
    rep.pop("_stage_ref", None)
    for key in ("f32_autograd", "f32_autograd_G", "f32_conditionals", "f32_conditionals_Gweighted"):
        print(key, json.dumps({k: f"{v:.2e}" for k, v in rep[key].items()}))
    if a.stages:
        print("f32 autograd stages", json.dumps({L: {k: f"{v:.2e}" for k, v in d.items()}
                                                 for L, d in rep["stages_f32_autograd"].items()}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
