"""The reference's demos/demo_tf2_2d_modified_multiclass.py (2-D inputs,
SMGPModified, MultiClass / RobustMax pred likelihood) run on the MI355X drop-in.

Differences from the reference script, all in the setup lines (the model,
training and prediction calls and the numpy post-processing are unchanged):
  * imports: `gpflow.kernels.SquaredExponential` -> `MixtureGPs.kernels`,
    `gpflow.likelihoods.MultiClass` / `RobustMax` -> `MixtureGPs.likelihoods`,
    `gpflow.utilities.print_summary` -> `MixtureGPs.utils`, `tf.data.Dataset`
    -> `utils.data.Dataset` (same from_tensor_slices/shuffle/batch/repeat
    pipeline); no TensorFlow import, so the two TF device prints and
    `tf.random.set_seed` become their torch counterparts;
  * plotting runs only with MGP_DEMO_PLOT=1 (matplotlib, Agg backend) and
    writes figs/demo_tf2_2d_modified_multiclass_1.png / _2.png next to this file; the
    plotting calls, interleaved with the prediction calls in the reference,
    sit under that switch, the prediction calls and numpy lines do not.
Run from the repository root: `python demos/demo_tf2_2d_modified_multiclass.py`.
The ELBO trajectory is the output the reference holds for this model
(final_figs/demo_tf2_2d_modified_multiclass_2.png, top-left panel); tests/test_gpu_demo.py checks
it against that band.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch
from scipy.cluster.vq import kmeans

from MixtureGPs.kernels import SquaredExponential
from MixtureGPs.likelihoods import GaussianModified, MultiClass, RobustMax
from MixtureGPs.models import SVGPModified, SMGPModified
from MixtureGPs.utils import print_summary
from utils.data import Dataset
from utils.dataset_utils import load_toy_2d_data_categorical
from utils.training_utils import run_adam

print(torch.cuda.is_available())
print("Num GPUs Available: ", torch.cuda.device_count())

PLOT = os.environ.get("MGP_DEMO_PLOT") == "1"
if PLOT:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.colors as mcolors
    from matplotlib import pyplot as plt

    colors = [mcolors.TABLEAU_COLORS[key] for key in mcolors.TABLEAU_COLORS.keys()]

seed = 0
torch.manual_seed(seed)
rng = np.random.default_rng(seed=seed)

N, Xtrain, Ytrain, Xtest = load_toy_2d_data_categorical(rng)

# Model configuration
num_iter = int(os.environ.get("MGP_DEMO_ITERS", 2000))  # Optimization iterations
lr = 0.005  # Learning rate for Adam opt
num_minibatch = 500  # Batch size for stochastic opt
num_samples = 25  # Number of MC samples
num_predict_samples = 100  # Number of prediction samples
num_data = Xtrain.shape[0]  # Training size
dimX = Xtrain.shape[1]  # Input dimensions
dimY = 1  # Output dimensions
num_ind = 25  # Inducing size for f
K = 2

input_dim = dimX
pred_kernel = SquaredExponential(variance=0.1, lengthscales=1.0)
assign_kernel = SquaredExponential(variance=0.1, lengthscales=1.0)
Z, Z_assign = kmeans(Xtrain, num_ind, seed=0)[0], kmeans(Xtrain, num_ind, seed=1)[0]

inv_link = RobustMax(num_classes=K)
lik = MultiClass(num_classes=K, invlink=inv_link)
assign_lik = GaussianModified(variance=0.5, D=K)

pred_layer = SVGPModified(kernel=pred_kernel, likelihood=lik, inducing_variable=Z, num_latent_gps=K,
                          whiten=True)
assign_layer = SVGPModified(kernel=assign_kernel, likelihood=assign_lik, inducing_variable=Z_assign, num_latent_gps=K,
                            whiten=True)

# model definition
model = SMGPModified(likelihood=lik, assign_likelihood=assign_lik, pred_layer=pred_layer,
                     assign_layer=assign_layer, K=K, num_samples=num_samples,
                     num_data=num_data)

print_summary(model)

dataset = Dataset.from_tensor_slices((Xtrain, Ytrain))
dataset = dataset.shuffle(buffer_size=num_data, seed=seed)
dataset = dataset.batch(num_minibatch).repeat()
train_iter = iter(dataset)

iters, elbos = run_adam(model, num_iter, train_iter, lr, compile=True)

print_summary(model)

n_batches = max(int(Xtrain.shape[0] / 500), 1)
Ss_y, Ss_f = [], []
for X_batch in np.array_split(Xtrain, n_batches):
    samples_y, samples_f = model.predict_samples(X_batch, S=num_predict_samples)
    Ss_y.append(samples_y)
    Ss_f.append(samples_f)
samples_y, samples_f = np.hstack(Ss_y), np.hstack(Ss_f)
mu_avg, fmu_avg = np.mean(samples_y, 0), np.mean(samples_f, 0)
samples_y_stack = np.reshape(samples_y, (num_predict_samples * Xtrain.shape[0], -1))
samples_f_stack = np.reshape(samples_f, (num_predict_samples * Xtrain.shape[0], -1))
Xt_tiled = np.tile(Xtrain, [num_predict_samples, 1])

if PLOT:
    fig_3d, fig = plt.figure(figsize=(14, 8)), plt.figure(figsize=(14, 8))
    ax_3d = [fig_3d.add_subplot(2, 2, i, projection='3d') for i in range(1, 5)]
    ax = [fig.add_subplot(2, 3, i) for i in range(1, 6)]
    ax_3d[0].scatter(Xtrain[:, 0], Xtrain[:, 1], Ytrain, s=1)
    ax_3d[1].scatter(Xt_tiled[:, 0:1], Xt_tiled[:, 1:2], samples_y_stack.flatten(), marker='+', alpha=0.01,
                     color=mcolors.TABLEAU_COLORS['tab:red'])
    ax_3d[1].scatter(Xt_tiled[:, 0:1], Xt_tiled[:, 1:2], samples_f_stack.flatten(), marker='+', alpha=0.01,
                     color=mcolors.TABLEAU_COLORS['tab:blue'])

assign_ = model.predict_assign(Xtrain)
if PLOT:
    for i in range(K):
        ax_3d[2].scatter(Xtrain[:, 0], Xtrain[:, 1], assign_[:, i], color=colors[i], s=1)

fmean, _ = model.predict_y(Xtrain)
fmean_ = np.mean(fmean, 0)
if PLOT:
    for i in range(K):
        ax_3d[3].scatter(Xtrain[:, 0], Xtrain[:, 1], fmean_[:, i], color=colors[i], s=1)
    ax[0].plot(iters, elbos, 'o-', ms=8, alpha=0.5)

stumpsX_const_value = 0.2
stumpsY_const_value = 0

Xtest_stumpsX = np.c_[Xtest[:, 0], stumpsY_const_value * np.ones(len(Xtest[:, 0]))]
Xtest_stumpsY = np.c_[stumpsX_const_value * np.ones(len(Xtest[:, 1])), Xtest[:, 1]]

Xtests = [Xtest_stumpsX, Xtest_stumpsY]

stump_assign, stump_fmean, stump_fvar = [], [], []
for i in range(2):
    assign_ = model.predict_assign(Xtests[i])
    stump_assign.append(assign_)
    if PLOT:
        ax[i + 1].plot(Xtests[i][:, i], assign_, 'o', markersize=1)

for i in range(2):
    fmean, fvar = model.predict_y(Xtests[i])
    fmean_, fvar_ = np.mean(fmean, 0), np.mean(fvar, 0)

    X_sorted = np.zeros_like(Xtests[i])
    sort_indices = np.argsort(Xtests[i][:, i])
    X_sorted[:, i] = Xtests[i][sort_indices, i]
    fmean_sorted = fmean_[sort_indices]
    fvar_sorted = fvar_[sort_indices]

    lb, ub = (fmean_sorted - 2 * fvar_sorted ** 0.5), (fmean_sorted + 2 * fvar_sorted ** 0.5)
    stump_fmean.append(fmean_sorted)
    stump_fvar.append(fvar_sorted)
    if PLOT:
        for k in range(K):
            ax[i + 3].plot(X_sorted[:, i], fmean_sorted[:, k], '-', alpha=1., color=colors[k])
            ax[i + 3].fill_between(X_sorted[:, i], lb[:, k], ub[:, k], alpha=0.3, color=colors[k])

if PLOT:
    plt.tight_layout()
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "figs")
    os.makedirs(out, exist_ok=True)
    fig_3d.savefig(os.path.join(out, "demo_tf2_2d_modified_multiclass_1.png"))
    fig.savefig(os.path.join(out, "demo_tf2_2d_modified_multiclass_2.png"))
