"""The five synthetic-data demo workloads of the reference, rebuilt as scenario
tests on the public drop-in API (no reference script text: each scenario is a
row of hyper-parameters, and one builder below turns a row into a model).

What the reference holds for these workloads is the ELBO-vs-iteration panel of
each figure under final_figs/ (float64 TF2 with TF's RNG).  The run
is stochastic (minibatch order, Monte-Carlo noise), so each trajectory is
checked against bands around the readings of its figure, and the predict_*
outputs are consumed by the same numpy operations a demo applies to them
(np.array_split batches -> np.hstack / np.mean / np.reshape / argmax).

Hyper-parameters, as data, from the demo scripts (setup lines):
  demo_tf2                          demos/demo_tf2.py:24-45,48,53-58
  demo_tf2_modified                 demos/demo_tf2_modified.py:24-51,53-60
  demo_tf2_modified_multiclass      demos/demo_tf2_modified_multiclass.py:22-51,53-60
  demo_tf2_2d                       demos/demo_tf2_2d.py:22-50,52-58
  demo_tf2_2d_modified_multiclass   demos/demo_tf2_2d_modified_multiclass.py:22-51,53-60
Figure readings (ELBO panel): final_figs/demo_tf2.png, demo_tf2_modified.png,
demo_tf2_modified_multiclass.png, demo_tf2_2d_2.png,
demo_tf2_2d_modified_multiclass_2.png.
"""
import numpy as np
import pytest
import torch
from scipy.cluster.vq import kmeans

from MixtureGPs.kernels import SquaredExponential
from MixtureGPs.likelihoods import GaussianModified, MultiClass, RobustMax
from MixtureGPs.models import SMGP, SMGPModified, SVGPModified
from MixtureGPs.utils import print_summary
from utils import dataset_utils
from utils.data import Dataset
from utils.training_utils import run_adam

pytestmark = pytest.mark.gpu

# one row per workload: data generator, model class, K, Adam iterations, kernel
# (variance, lengthscale) of each layer, likelihoods, what the predictions run on,
# and the ELBO bands (iteration window -> (lo, hi); "mean"/"median" over the window)
SCENARIOS = {
    "demo_tf2": dict(
        data="load_toy_multimodal_data", model="SMGP", K=3, iters=2000,
        pred_kernel=(0.5, 0.5), assign_kernel=(0.1, 1.0), lik=("gauss", 0.5), assign_lik=None,
        samples_on="test", assign_on="train", predict_on="test", stumps=None, plot_draw=None,
        stat="mean",
        # readings: -2.85 @5, -1.4 @500, -0.7 @1000, -0.1 @2000
        bands={(5, 5): (-3.4, -2.3), (450, 550): (-1.8, -1.0), (950, 1050): (-1.1, -0.35),
               (1900, 2000): (-0.4, 0.15)}),
    "demo_tf2_modified": dict(
        data="load_toy_multimodal_data", model="SMGPModified", K=3, iters=4000,
        pred_kernel=(0.5, 0.5), assign_kernel=(0.1, 1.0), lik=("gauss", 0.5), assign_lik=("gauss", 0.5),
        samples_on="test", assign_on="train", predict_on="test", stumps=None, plot_draw=None,
        stat="mean",
        # readings: -5.2 @5, plateau -2.8 (250-800), -1.0 @2000, -1.0 to 4000; the
        # escape from the plateau (~1000) is the stochastic part and is not banded
        bands={(5, 5): (-6.2, -4.0), (450, 550): (-3.4, -2.2), (1900, 2100): (-1.8, -0.5),
               (3500, 4000): (-1.5, -0.5)}),
    "demo_tf2_modified_multiclass": dict(
        data="load_toy_data_categorical", model="SMGPModified", K=2, iters=2000,
        pred_kernel=(0.1, 1.0), assign_kernel=(0.1, 1.0), lik=("multiclass",), assign_lik=("gauss", 0.5),
        samples_on="plot", assign_on="train", predict_on="test", stumps=None, plot_draw=(200, 2.0),
        stat="median",
        # readings: -4.4 @5, -0.6 @500, +0.6 @1000, +1.4 @2000 (isolated dips -> medians)
        bands={(5, 5): (-5.4, -3.4), (450, 550): (-1.4, 0.2), (950, 1050): (-0.3, 1.3),
               (1900, 2000): (0.7, 2.0)}),
    "demo_tf2_2d": dict(
        data="load_toy_2d_data", model="SMGP", K=3, iters=2000,
        pred_kernel=(0.1, 1.0), assign_kernel=(0.1, 1.0), lik=("gauss", 0.5), assign_lik=None,
        samples_on="train", assign_on="train", predict_on="train", stumps=(-0.25, 0.75), plot_draw=None,
        stat="median",
        # readings: -228 @5, -25 @500, -2 from 1500 to 2000
        bands={(5, 5): (-270, -190), (450, 550): (-50, -10), (1900, 2000): (-8, 0.5)}),
    "demo_tf2_2d_modified_multiclass": dict(
        data="load_toy_2d_data_categorical", model="SMGPModified", K=2, iters=2000,
        pred_kernel=(0.1, 1.0), assign_kernel=(0.1, 1.0), lik=("multiclass",), assign_lik=("gauss", 0.5),
        samples_on="train", assign_on="train", predict_on="train", stumps=(0.2, 0.0), plot_draw=None,
        stat="median",
        # readings: -4.3 @5, -1.1 @500, 0.0 @1000, +1.05 @2000
        bands={(5, 5): (-5.2, -3.4), (450, 550): (-1.7, -0.5), (950, 1050): (-0.8, 0.8),
               (1900, 2000): (0.4, 1.8)}),
}

# settings every workload shares (the demos' module constants)
COMMON = dict(seed=0, lr=0.005, batch=500, S=25, predict_S=100, num_inducing=25)


def _likelihood(spec, K, device):
    if spec[0] == "gauss":
        return GaussianModified(variance=spec[1], D=K, device=device)
    return MultiClass(num_classes=K, invlink=RobustMax(num_classes=K))


def run_scenario(name, device):
    """Build the workload `name` through the drop-in API, train it with run_adam,
    and evaluate its predictions the way the demos consume them."""
    sc, c = SCENARIOS[name], COMMON
    torch.manual_seed(c["seed"])
    rng = np.random.default_rng(seed=c["seed"])
    num_data, Xtrain, Ytrain, Xtest = getattr(dataset_utils, sc["data"])(rng)
    num_data = Xtrain.shape[0]
    inputs = {"train": Xtrain, "test": Xtest}
    if sc["plot_draw"] is not None:   # an extra grid drawn from the same generator
        n_plot, margin = sc["plot_draw"]
        inputs["plot"] = rng.uniform(Xtrain[:, 0].min() - margin, Xtrain[:, 0].max() + margin, (n_plot, 1))
    K = sc["K"]
    Zs = [kmeans(Xtrain, c["num_inducing"], seed=s)[0] for s in (0, 1)]
    lik = _likelihood(sc["lik"], K, device)
    assign_lik = _likelihood(sc["assign_lik"], K, device) if sc["assign_lik"] else lik
    layers = [SVGPModified(kernel=SquaredExponential(variance=v, lengthscales=ls), likelihood=l,
                           inducing_variable=Z, num_latent_gps=K, whiten=True)
              for (v, ls), l, Z in ((sc["pred_kernel"], lik, Zs[0]), (sc["assign_kernel"], assign_lik, Zs[1]))]
    common = dict(pred_layer=layers[0], assign_layer=layers[1], K=K, num_samples=c["S"], num_data=num_data)
    if sc["model"] == "SMGP":
        model = SMGP(likelihood=lik, **common)
    else:
        model = SMGPModified(likelihood=lik, assign_likelihood=assign_lik, **common)
    print_summary(model)
    ds = Dataset.from_tensor_slices((Xtrain, Ytrain)).shuffle(buffer_size=num_data, seed=c["seed"])
    iters, elbos = run_adam(model, sc["iters"], iter(ds.batch(c["batch"]).repeat()), c["lr"])

    out = {"iters": iters, "elbos": elbos, "Xtrain": Xtrain}
    Xs = inputs[sc["samples_on"]]
    parts = [model.predict_samples(xb, S=c["predict_S"])
             for xb in np.array_split(Xs, max(Xs.shape[0] // 500, 1))]
    sy, sf = np.hstack([p[0] for p in parts]), np.hstack([p[1] for p in parts])
    out.update(samples_y=sy, samples_f=sf, n_samples_x=Xs.shape[0], mu_avg=np.mean(sy, 0),
               y_stack=np.reshape(sy, (c["predict_S"] * Xs.shape[0], -1)))
    out["assign"] = model.predict_assign(inputs[sc["assign_on"]])
    out["labels"] = np.argmax(out["assign"], 1)
    Xp = inputs[sc["predict_on"]]
    fmean, fvar = model.predict_y(Xp)
    out.update(fmean_=np.mean(fmean, 0), fvar_=np.mean(fvar, 0), n_predict=Xp.shape[0])
    if sc["stumps"] is not None:    # slices through the 2-D input at a fixed other coordinate
        x_fix, y_fix = sc["stumps"]
        slices = [np.c_[Xtest[:, 0], np.full(len(Xtest), y_fix)], np.c_[np.full(len(Xtest), x_fix), Xtest[:, 1]]]
        out["stumps"] = []
        for i, Xsl in enumerate(slices):
            a = model.predict_assign(Xsl)
            m, v = model.predict_y(Xsl)
            order = np.argsort(Xsl[:, i])
            out["stumps"].append((a, np.mean(m, 0)[order], np.mean(v, 0)[order]))
        out["n_test"] = Xtest.shape[0]
    return out


def _window(iters, elbos, lo, hi, stat):
    v = [e for i, e in zip(iters, elbos) if lo <= i <= hi]
    assert v, (lo, hi)
    return float(np.median(v) if stat == "median" else np.mean(v))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", list(SCENARIOS))
def test_scenario(device, name):
    sc = SCENARIOS[name]
    r = run_scenario(name, device)
    iters, elbos = r["iters"], r["elbos"]
    # run_adam's record: every 5th iteration (utils/training_utils.py:19-23)
    assert iters[0] == 5 and iters[-1] == sc["iters"] and len(iters) == sc["iters"] // 5
    assert np.all(np.isfinite(elbos))
    got = {w: _window(iters, elbos, *w, sc["stat"]) for w in sc["bands"]}
    print(name, " ".join(f"{w[0]}-{w[1]}: {g:.3f}" for w, g in got.items()))
    for w, (lo, hi) in sc["bands"].items():
        assert lo < got[w] < hi, (name, w, got[w], (lo, hi))
    K, P = sc["K"], COMMON["predict_S"]
    assert r["samples_y"].shape == (P, r["n_samples_x"], 1) and r["samples_f"].shape == r["samples_y"].shape
    assert r["mu_avg"].shape == (r["n_samples_x"], 1) and r["y_stack"].shape == (P * r["n_samples_x"], 1)
    assert np.all(np.isfinite(r["samples_y"]))
    n_assign = r["Xtrain"].shape[0]
    assert r["assign"].shape == (n_assign, K) and np.allclose(r["assign"].sum(1), 1.0, atol=1e-5)
    assert r["labels"].shape == (n_assign,)
    assert r["fmean_"].shape == (r["n_predict"], K) and np.all(r["fvar_"] >= 0)
    for a, fm, fv in r.get("stumps", []):
        assert a.shape == (r["n_test"], K) and np.allclose(a.sum(1), 1.0, atol=1e-5)
        assert fm.shape == (r["n_test"], K) and np.all(fv >= 0)
