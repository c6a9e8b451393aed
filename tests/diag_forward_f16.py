"""Forward-conditional accuracy per layer and variant (diagnostic, not collected by pytest).

    python -m tests.diag_forward_f16 [--N 65536 --M 1024 --K 8 --D 8 --ls 1.0]

Test infrastructure (imports oracle/ as the checker).  For the c3 problem it compares
each layer's (fmean, fvar) from SMGP.conditionals against the float64 oracle
(cpu_ref.svgp_predict_f_dedup, models.py:129-144), normwise, for the split-f16 chain
(default), the x6 chain, the split-f16 chain with the layers' kernel variances swapped,
with K1 as its own launches (schedule "overlap") and with per-layer K4 / K5 launches.
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
from tests.helpers import build_model, normwise, to_np   # noqa: E402


def oracle(X, p):
    out = {}
    for name, L in (("f", p.pred), ("a", p.assign)):
        f32 = lambda v: np.asarray(v, np.float64).astype(np.float32).astype(np.float64)
        fm, fv = R.svgp_predict_f_dedup(f32(X), f32(L["Z"]), f32(L["variance"]), f32(L["lengthscales"]),
                                        f32(L["q_mu"]), f32(L["q_sqrt"]))
        out["mu_" + name], out["var_" + name] = fm.T, fv.T
    return out


def run(p, X, device, a):
    model = build_model(p, device)
    cond = model.conditionals(torch.as_tensor(X, dtype=torch.float32, device=device))
    torch.cuda.synchronize()
    return {k: to_np(c)[:, :a.N] for k, c in zip(("mu_f", "var_f", "mu_a", "var_a"), cond)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--M", type=int, default=1024)
    ap.add_argument("--K", type=int, default=8)
    ap.add_argument("--D", type=int, default=8)
    ap.add_argument("--ls", type=float, default=1.0)
    ap.add_argument("--variants", default="f16,x6,swap,overlap,unbatched,var05")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from modulatedgps_amd import config, models
    device = torch.device("cuda", 0)
    t0 = time.time()
    X, Y, p = R.synthetic_problem(a.N, a.M, a.K, a.D, a.ls, state="perturbed", S=5)
    refs = {"base": oracle(X, p)}
    print(f"oracle {time.time() - t0:.0f}s", flush=True)
    rep = {}
    for v in a.variants.split(","):
        pp, key = p, "base"
        if v == "swap":
            X2, Y2, pp = R.synthetic_problem(a.N, a.M, a.K, a.D, a.ls, state="perturbed", S=5,
                                             var_pred=0.1, var_assign=0.5)
            key = "swap"
        elif v == "var05":
            X2, Y2, pp = R.synthetic_problem(a.N, a.M, a.K, a.D, a.ls, state="perturbed", S=5,
                                             var_pred=0.5, var_assign=0.5)
            key = "var05"
        elif v.startswith("var="):   # var=<pred>/<assign>[/x6]
            vp, va = (float(x) for x in v[4:].split("/")[:2])
            X2, Y2, pp = R.synthetic_problem(a.N, a.M, a.K, a.D, a.ls, state="perturbed", S=5,
                                             var_pred=vp, var_assign=va)
            key = f"var={vp}/{va}"
        if key not in refs:
            refs[key] = oracle(X, pp)
            print(f"oracle {key} {time.time() - t0:.0f}s", flush=True)
        old = (config.expert_format(), config.step_schedule(), models._K4_BATCHED)
        try:
            config.set_expert_format("x6" if v == "x6" or v.endswith("/x6") else "f16")
            if v == "overlap":
                config.set_step_schedule("overlap")
            if v == "unbatched":
                models._K4_BATCHED = False
            got = run(pp, X, device, a)
        finally:
            config.set_expert_format(old[0])
            config.set_step_schedule(old[1])
            models._K4_BATCHED = old[2]
        rep[v] = {k: normwise(got[k], refs[key][k]) for k in got}
        for k in got:
            err = np.abs(got[k] - refs[key][k])
            rep[v][k + "_maxabs_over_maxref"] = float(err.max() / np.abs(refs[key][k]).max())
        print(v, json.dumps({k: f"{e:.2e}" for k, e in rep[v].items()}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rep, f, indent=1)


if __name__ == "__main__":
    main()
