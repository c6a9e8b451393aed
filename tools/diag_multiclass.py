"""Diagnostic: run the demo_tf2_modified_multiclass training loop and stop at
the first step whose gradient or parameters are non-finite, printing which
blocks and the layers' minimum marginal variance on that batch.
Run on the GPU box from the repo root: python tools/diag_multiclass.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from scipy.cluster.vq import kmeans  # noqa: E402

from MixtureGPs.kernels import SquaredExponential  # noqa: E402
from MixtureGPs.likelihoods import GaussianModified, MultiClass, RobustMax  # noqa: E402
from MixtureGPs.models import SVGPModified, SMGPModified  # noqa: E402
from modulatedgps_amd.training import AdamTF  # noqa: E402
from utils.data import Dataset  # noqa: E402
from utils.dataset_utils import load_toy_data_categorical  # noqa: E402

torch.manual_seed(0)
rng = np.random.default_rng(seed=0)
N, Xtrain, Ytrain, Xtest = load_toy_data_categorical(rng)
K = 2
Z, Z_assign = kmeans(Xtrain, 25, seed=0)[0], kmeans(Xtrain, 25, seed=1)[0]
lik = MultiClass(num_classes=K, invlink=RobustMax(num_classes=K))
assign_lik = GaussianModified(variance=0.5, D=K)
pred_layer = SVGPModified(kernel=SquaredExponential(variance=0.1, lengthscales=1.0), likelihood=lik,
                          inducing_variable=Z, num_latent_gps=K, whiten=True)
assign_layer = SVGPModified(kernel=SquaredExponential(variance=0.1, lengthscales=1.0), likelihood=assign_lik,
                            inducing_variable=Z_assign, num_latent_gps=K, whiten=True)
model = SMGPModified(likelihood=lik, assign_likelihood=assign_lik, pred_layer=pred_layer,
                     assign_layer=assign_layer, K=K, num_samples=25, num_data=Xtrain.shape[0])
ds = Dataset.from_tensor_slices((Xtrain, Ytrain)).shuffle(buffer_size=Xtrain.shape[0], seed=0).batch(500).repeat()
it = iter(ds)
opt = AdamTF(model.trainable_parameters(), 0.005)
params = {name: theta for name, theta, _ in opt.params}
for i in range(1, int(os.environ.get("DIAG_ITERS", 2000)) + 1):
    X, Y = next(it)
    elbo, grads = model.elbo_and_grad(X, Y)
    bad = [n for n, g in grads.items() if not torch.isfinite(g).all()]
    if bad or not torch.isfinite(elbo).all():
        print(f"iter {i}: elbo {float(elbo):.4f}, non-finite gradient blocks: {bad}")
        for layer_name, layer in (("pred", pred_layer), ("assign", assign_layer)):
            fm, fv = layer.predict_f(X)
            fv = fv.detach().float()
            print(f"  {layer_name}: fvar min {float(fv.min()):.3e} max {float(fv.max()):.3e}, "
                  f"n(fvar<0) {int((fv < 0).sum())}, n(fvar<-1e-6) {int((fv < -1e-6).sum())}")
        for n, t in params.items():
            if t.numel() <= 4:
                print(f"  param {n} = {t.detach().cpu().numpy().ravel()}")
        for n in bad:
            g = grads[n]
            print(f"  grad {n}: n_nonfinite {int((~torch.isfinite(g)).sum())} of {g.numel()}")
        sys.exit(0)
    opt.step(grads)
    if i % 100 == 0:
        fmins = []
        for layer in (pred_layer, assign_layer):
            fv = layer.predict_f(X)[1].detach().float()
            fmins.append(float(fv.min()))
        print(f"iter {i}: elbo {float(elbo):.4f} fvar min pred {fmins[0]:.3e} assign {fmins[1]:.3e}", flush=True)
print("no non-finite step")
