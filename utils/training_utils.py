"""Drop-in for the reference's utils/training_utils.py (run_adam, :4-28).

Same signature and return value: run_adam(model, num_iter, train_iter, lr,
compile=True) -> (iters, elbos).  Each iteration draws a batch from train_iter
and runs one optimisation step (forward + backward + TF-legacy Adam, all on the
HIP kernels); every 5th iteration the ELBO of a further batch is evaluated and
recorded, as the reference does (:15-23).  At that readback a failed Cholesky of
Kuu (K3's info != 0, e.g. after a step that made Kuu indefinite) raises
MGPLinAlgError, where the reference raises InvalidArgumentError from
base_conditional (MixtureGPs/models.py:141); a NaN parameter keeps the pivot
non-positive, so a failure between readbacks is still reported.  `compile` is
accepted for API compatibility (the step is a fixed sequence of kernel launches)."""
import numpy as np

from modulatedgps_amd.training import AdamTF


def run_adam(model, num_iter, train_iter, lr, compile=True):
    optimizer = AdamTF(model.trainable_parameters(), lr)

    def optimization_step():
        X, Y = next(train_iter)
        _, grads = model.elbo_and_grad(np.asarray(X) if not hasattr(X, "device") else X,
                                       np.asarray(Y) if not hasattr(Y, "device") else Y)
        optimizer.step(grads)

    print('{:>5s}'.format("iter") + '{:>24s}'.format("ELBO:"))
    iters = []
    elbos = []
    for i in range(1, num_iter + 1):
        try:
            optimization_step()
            if i % 5 == 0 or i == 0:
                elbo = -float(model.training_loss(next(train_iter)).cpu())
                if hasattr(model, "check_linalg"):
                    model.check_linalg()  # a failed Cholesky raises here (models.py:141)
                print('{:>5d}'.format(i) + '{:>24.6f}'.format(elbo))
                iters.append(i)
                elbos.append(elbo)
        except KeyboardInterrupt:
            print("stopping training")
            break
    return iters, elbos
