"""The reference's demos/demo_tf2_modified.py (SMGPModified) run on the MI355X drop-in.

Differences from the reference script, all in the setup lines (the model,
training and prediction calls and the numpy post-processing are unchanged):
  * imports: `gpflow.kernels.SquaredExponential` -> `MixtureGPs.kernels`,
    `gpflow.utilities.print_summary` -> `MixtureGPs.utils`, `tf.data.Dataset`
    -> `utils.data.Dataset` (same from_tensor_slices/shuffle/batch/repeat
    pipeline); no TensorFlow import, so the two TF device prints and
    `tf.random.set_seed` become their torch counterparts;
  * plotting runs only with MGP_DEMO_PLOT=1 (matplotlib, Agg backend) and
    writes figs/demo_tf2_modified.png next to this file.
Run from the repository root: `python demos/demo_tf2_modified.py`.  The ELBO
trajectory is the output the reference holds for this model
(final_figs/demo_tf2_modified.png, top-right panel); tests/test_gpu_demo.py
checks it against that band.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch
from scipy.cluster.vq import kmeans

from MixtureGPs.kernels import SquaredExponential
from MixtureGPs.likelihoods import GaussianModified
from MixtureGPs.models import SVGPModified, SMGPModified
from MixtureGPs.utils import print_summary
from utils.data import Dataset
from utils.dataset_utils import load_toy_multimodal_data
from utils.training_utils import run_adam

print(torch.cuda.is_available())
print("Num GPUs Available: ", torch.cuda.device_count())

seed = 0
torch.manual_seed(seed)
rng = np.random.default_rng(seed=seed)

N, Xtrain, Ytrain, Xtest = load_toy_multimodal_data(rng)

# Model configuration
num_iter = int(os.environ.get("MGP_DEMO_ITERS", 4000))  # Optimization iterations
lr = 0.005  # Learning rate for Adam opt
num_minibatch = 500  # Batch size for stochastic opt
num_samples = 25  # Number of MC samples
num_predict_samples = 100  # Number of prediction samples
num_data = Xtrain.shape[0]  # Training size
dimX = Xtrain.shape[1]  # Input dimensions
dimY = 1  # Output dimensions
num_ind = 25  # Inducing size for f
K = 3

input_dim = dimX
pred_kernel = SquaredExponential(variance=0.5, lengthscales=0.5)
assign_kernel = SquaredExponential(variance=0.1, lengthscales=1.0)
Z, Z_assign = kmeans(Xtrain, num_ind, seed=0)[0], kmeans(Xtrain, num_ind, seed=1)[0]

lik = GaussianModified(variance=0.5, D=K)
assign_lik = GaussianModified(variance=0.5, D=K)

pred_layer = SVGPModified(kernel=pred_kernel, likelihood=lik, inducing_variable=Z, num_latent_gps=K, whiten=True)
assign_layer = SVGPModified(kernel=assign_kernel, likelihood=assign_lik, inducing_variable=Z_assign, num_latent_gps=K,
                            whiten=True)

# model definition
model = SMGPModified(likelihood=lik, assign_likelihood=assign_lik, pred_layer=pred_layer, assign_layer=assign_layer,
                     K=K, num_samples=num_samples,
                     num_data=num_data)

print_summary(model)

dataset = Dataset.from_tensor_slices((Xtrain, Ytrain))
dataset = dataset.shuffle(buffer_size=num_data, seed=seed)
dataset = dataset.batch(num_minibatch).repeat()
train_iter = iter(dataset)

iters, elbos = run_adam(model, num_iter, train_iter, lr, compile=True)

print_summary(model)

n_batches = max(int(Xtest.shape[0] / 500), 1)
Ss_y, Ss_f = [], []
for X_batch in np.array_split(Xtest, n_batches):
    samples_y, samples_f = model.predict_samples(X_batch, S=num_predict_samples)
    Ss_y.append(samples_y)
    Ss_f.append(samples_f)
samples_y, samples_f = np.hstack(Ss_y), np.hstack(Ss_f)
mu_avg, fmu_avg = np.mean(samples_y, 0), np.mean(samples_f, 0)
samples_y_stack = np.reshape(samples_y, (num_predict_samples * Xtest.shape[0], -1))
samples_f_stack = np.reshape(samples_f, (num_predict_samples * Xtest.shape[0], -1))
Xt_tiled = np.tile(Xtest, [num_predict_samples, 1])

assign_ = model.predict_assign(Xtrain)

fmean, fvar = model.predict_y(Xtest)
fmean_, fvar_ = np.mean(fmean, 0), np.mean(fvar, 0)
lb, ub = (fmean_ - 2 * fvar_ ** 0.5), (fmean_ + 2 * fvar_ ** 0.5)
I = np.argmax(assign_, 1)

if os.environ.get("MGP_DEMO_PLOT") == "1":
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.colors as mcolors
    from matplotlib import pyplot as plt

    colors = [mcolors.TABLEAU_COLORS[key] for key in mcolors.TABLEAU_COLORS.keys()]
    f, ax = plt.subplots(2, 2, figsize=(14, 8))
    ax[0, 0].scatter(Xt_tiled.flatten(), samples_y_stack.flatten(), marker='+', alpha=0.01,
                     color=mcolors.TABLEAU_COLORS['tab:red'])
    ax[0, 0].scatter(Xt_tiled.flatten(), samples_f_stack.flatten(), marker='+', alpha=0.01,
                     color=mcolors.TABLEAU_COLORS['tab:blue'])
    ax[0, 0].scatter(Xtrain, Ytrain, marker='x', color='black', alpha=0.1)
    ax[0, 0].set_title("Many GPs")
    ax[0, 1].plot(iters, elbos, 'o-', ms=8, alpha=0.5)
    ax[0, 1].set_xlabel('Iterations')
    ax[0, 1].set_ylabel('ELBO')
    ax[1, 0].plot(Xtrain, assign_, 'o')
    ax[1, 0].set_ylabel('softmax(assignment)')
    for i in range(K):
        ax[1, 1].plot(Xtest.flatten(), fmean_[:, i], '-', alpha=1., color=colors[i])
        ax[1, 1].fill_between(Xtest.flatten(), lb[:, i], ub[:, i], alpha=0.3, color=colors[i])
    ax[1, 1].scatter(Xtrain, Ytrain, marker='x', color='black', alpha=0.5)
    plt.tight_layout()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "figs")
    os.makedirs(out, exist_ok=True)
    plt.savefig(os.path.join(out, "demo_tf2_modified.png"))
