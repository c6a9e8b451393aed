"""Generate the golden fixtures under tests/golden/ (run in the build container).

    python tests/golden/make_golden.py [--reference /root/reference]

* ``demo_tf2_data.npz``: the demo_tf2 training data produced by the REFERENCE'S
  OWN generator ``utils/dataset_utils.py:100-114`` (``load_toy_multimodal_data``
  with ``np.random.default_rng(0)``, exactly as ``demos/demo_tf2.py:17-21``), plus
  the kmeans inducing points of ``demos/demo_tf2.py:39`` (scipy kmeans, seeds 0/1,
  stored because scipy here is 1.15 not the pinned 1.10).  Only the arrays are
  committed; no reference source travels.
* ``toy_datasets.npz``: the outputs of the reference's other toy generators
  (``utils/dataset_utils.py:84-166``) that the demos load, pinning the drop-in
  ``utils/dataset_utils.py``.
* ``case_*.npz``: inputs, parameters, explicit noise and the float64 oracle
  outputs (ELBO, KL, per-layer fmean/fvar, predict_y, predict_assign) for the
  parity tests.  Large inputs (the c2-shaped case) are not stored: the test
  regenerates them with ``oracle.cpu_ref.synthetic_problem`` (seeded PCG64) and
  the fixture pins the outputs.

TensorFlow/GPflow are not importable here, so the outputs come from the
oracle restatement ("parity unpinned, identity-pinned": see oracle/cpu_ref.py).
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import cpu_ref as R  # noqa: E402
from oracle import philox  # noqa: E402


def demo_data(reference):
    sys.path.insert(0, reference)
    from utils.dataset_utils import load_toy_multimodal_data  # reference's own generator
    from scipy.cluster.vq import kmeans
    rng = np.random.default_rng(seed=0)                       # demo_tf2.py:17-18
    N, Xtrain, Ytrain, Xtest = load_toy_multimodal_data(rng)  # demo_tf2.py:20
    Z = kmeans(Xtrain, 25, seed=0)[0]                          # demo_tf2.py:39
    Z_assign = kmeans(Xtrain, 25, seed=1)[0]
    Z20 = kmeans(Xtrain[:600], 20, seed=0)[0]
    Z20_assign = kmeans(Xtrain[:600], 20, seed=1)[0]
    return dict(N=N, Xtrain=Xtrain, Ytrain=Ytrain, Xtest=Xtest, Z=Z, Z_assign=Z_assign,
                Z20=Z20, Z20_assign=Z20_assign)


def toy_datasets(reference):
    """Outputs of the reference's own toy generators (utils/dataset_utils.py:84-166):
    numpy Generator seed 0 for the Generator-based ones, np.random.seed(0) for the
    global-RNG association set.  Arrays only; no reference source is stored."""
    sys.path.insert(0, reference)
    from utils import dataset_utils as U
    out = {}
    for name in ("load_toy_data_categorical", "load_toy_multimodal_data", "load_toy_2d_data",
                 "load_toy_2d_data_categorical"):
        N, X, Y, Xt = getattr(U, name)(np.random.default_rng(0))
        out.update({f"{name}_N": N, f"{name}_X": X, f"{name}_Y": Y, f"{name}_Xtest": Xt})
    np.random.seed(0)
    N, X, Y, Xt = U.load_toy_data_assoc()
    out.update({"load_toy_data_assoc_N": N, "load_toy_data_assoc_X": X, "load_toy_data_assoc_Y": Y,
                "load_toy_data_assoc_Xtest": Xt})
    return out


def perturbed_layer(Z, var, ls, K, rng):
    M = Z.shape[0]
    return dict(Z=Z, variance=var, lengthscales=ls, q_mu=0.5 * rng.standard_normal((M, K)),
                q_sqrt=0.5 * np.eye(M)[None] + np.tril(0.1 * rng.standard_normal((K, M, M))))


def init_layer(Z, var, ls, K):
    M = Z.shape[0]
    return dict(Z=Z, variance=var, lengthscales=ls, q_mu=np.zeros((M, K)),
                q_sqrt=np.tile(np.eye(M)[None], (K, 1, 1)))


def outputs(X, Y, p, z, u, Xtest, seed):
    elbo, parts = R.smgp_elbo(X, Y, p, z, u, return_parts=True)
    zp = philox.noise_normal(seed, p.S, np.arange(X.shape[0]), p.lik_variance.shape[1])
    up = philox.noise_uniform(seed, p.S, np.arange(X.shape[0]), p.lik_variance.shape[1])
    elbo_philox = R.smgp_elbo(X, Y, p, zp, up)
    my, vy = R.predict_y(Xtest, p)
    pa = R.predict_assign(Xtest, p)
    return dict(elbo=elbo, elbo_philox=elbo_philox, philox_seed=seed,
                data_term=parts["data_term"], kl_f=parts["kl_f"], kl_a=parts["kl_a"],
                mu_f=parts["mu_f"], var_f=parts["var_f"], mu_a=parts["mu_a"], var_a=parts["var_a"],
                predict_y_mean=my, predict_y_var=vy, predict_assign=pa)


def pack(X, Y, p, z, u, Xtest, out, store_inputs=True, extra=None):
    d = dict(S=p.S, num_data=p.num_data, lik_variance=p.lik_variance, **out)
    if store_inputs:
        d.update(X=X, Y=Y, Xtest=Xtest, z=z, u=u)
        for name, L in (("pred", p.pred), ("assign", p.assign)):
            for key, val in L.items():
                d[f"{name}_{key}"] = np.asarray(val)
    if extra:
        d.update(extra)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", choices=("all", "toy"), default="all",
                    help="toy: regenerate only toy_datasets.npz")
    args = ap.parse_args()
    np.savez_compressed(os.path.join(HERE, "toy_datasets.npz"), **toy_datasets(args.reference))
    if args.only == "toy":
        return
    dd = demo_data(args.reference)
    np.savez_compressed(os.path.join(HERE, "demo_tf2_data.npz"), **dd)

    S, K = 25, 3
    Xb, Yb = dd["Xtrain"][:500], dd["Ytrain"][:500]           # one batch of 500 (demo_tf2.py:26)
    Xtest = dd["Xtest"]
    # demo_tf2 shapes, SVGP init state (demo_tf2.py:37-48)
    p = R.SMGPParams(init_layer(dd["Z"], 0.5, 0.5, K), init_layer(dd["Z_assign"], 0.1, 1.0, K),
                     0.5 * np.ones((1, K)), num_data=dd["N"], S=S)
    z, u = R.explicit_noise(S, 500, K, seed=5)
    out = outputs(Xb, Yb, p, z, u, Xtest, seed=1234)
    out["elbo_faithful"] = R.smgp_elbo(Xb, Yb, p, z, u, faithful=True)
    np.savez_compressed(os.path.join(HERE, "case_demo_init.npz"), **pack(Xb, Yb, p, z, u, Xtest, out))

    # demo_tf2 shapes, perturbed variational state
    r = np.random.default_rng(4)
    p = R.SMGPParams(perturbed_layer(dd["Z"], 0.5, 0.5, K, r),
                     perturbed_layer(dd["Z_assign"], 0.1, 1.0, K, r),
                     np.array([[0.3, 0.5, 0.8]]), num_data=dd["N"], S=S)
    out = outputs(Xb, Yb, p, z, u, Xtest, seed=1234)
    out["elbo_faithful"] = R.smgp_elbo(Xb, Yb, p, z, u, faithful=True)
    np.savez_compressed(os.path.join(HERE, "case_demo_perturbed.npz"),
                        **pack(Xb, Yb, p, z, u, Xtest, out))

    # BASELINE config 1: N=600, M=20, K=3, D=1 (demo_tf2 data, kmeans-20 Z)
    X1, Y1 = dd["Xtrain"][:600], dd["Ytrain"][:600]
    r = np.random.default_rng(14)
    p = R.SMGPParams(perturbed_layer(dd["Z20"], 0.5, 0.5, K, r),
                     perturbed_layer(dd["Z20_assign"], 0.1, 1.0, K, r),
                     0.5 * np.ones((1, K)), num_data=600, S=S)
    z, u = R.explicit_noise(S, 600, K, seed=15)
    out = outputs(X1, Y1, p, z, u, Xtest, seed=77)
    np.savez_compressed(os.path.join(HERE, "case_c1.npz"), **pack(X1, Y1, p, z, u, Xtest, out))

    # BASELINE config 2 shapes (M=256, K=4, D=2, l=0.15) at reduced N=1024: outputs only
    gen = dict(N=1024, M=256, K=4, D=2, ls_pred=0.15, state="perturbed", S=25, seed=0)
    X2, Y2, p = R.synthetic_problem(**gen)
    z, u = R.explicit_noise(25, 1024, 4, seed=5)
    Xt2 = X2[:128]
    out = outputs(X2, Y2, p, z, u, Xt2, seed=99)
    extra = {f"gen_{k}": np.asarray(v) for k, v in gen.items()}
    np.savez_compressed(os.path.join(HERE, "case_c2r.npz"),
                        **pack(X2, Y2, p, z, u, Xt2, out, store_inputs=False, extra=extra))
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
