"""Block-level simulation (numpy, float64) of K3's launch sequence with the look-ahead row
preparation (chol.hip, round 5): chol_prep, step launches j = 0 .. nb-2 (look-ahead of tile
j+1, RowPrep of row j+2, the pairs' tiles with the lead rows j+1 / j+2), chol_last_step.
Checks L and L^-1 against numpy.  Usage: python tools/k3_blocked_sim.py"""
import numpy as np


def chol_inv(A):
    L = np.linalg.cholesky(A)
    return L, np.linalg.inv(L)


def simulate(Kuu, nb, B=64):
    T = lambda X, i, l: X[i * B:(i + 1) * B, l * B:(l + 1) * B]
    W = {(i, l): T(Kuu, i, l).copy() for i in range(nb) for l in range(i + 1)}
    Bt = {}                      # forward-substitution tiles B_ic (start: identity blocks, implicit)
    D, LS, Lout, X = {}, {}, {}, {}
    # prep: factor tile 0
    L00, D[0] = chol_inv(W[0, 0])
    Lout[0, 0] = L00
    for j in range(nb - 1):
        s, r = j + 1, j + 2
        # look-ahead group 0: tile s
        if j == 0:
            P = W[s, j] @ D[j].T
            LS[0] = P
            F = W[s, s] - P @ P.T
        else:
            F = W[s, s]          # prepared by the previous launch's RowPrep
        Lss, Ds = chol_inv(F)
        # RowPrep (group 1): row r
        if r < nb:
            Lrj = W[r, j] @ D[j].T
            Wrs = W[r, s] - Lrj @ LS[j].T
            Frr = W[r, r] - Lrj @ Lrj.T
            Lrs = Wrs @ np.linalg.inv(Lss).T     # progressive TRSM (column blocks of 16 in HIP)
            Frr = Frr - Lrs @ Lrs.T
            LS[j + 1] = Lrs
            W[r, r] = Frr
        # pairs: rows i = j+1 .. nb-1
        Pi = {}
        for i in range(j + 1, nb):
            Pi[i] = LS[j] if (j >= 1 and i == j + 1) else W[i, j] @ D[j].T
        Lout.update({(i, j): Pi[i] for i in range(j + 1, nb)})
        for i in range(j + 1, nb):
            lead = i <= j + 2
            if not lead:
                for l in range(j + 1, i + 1):        # update tiles incl. the diagonal
                    W[i, l] = W[i, l] - Pi[i] @ Pi[l].T
            # forward substitution: X_jc = D_j B_jc (c < j), X_jj = D_j; B_ic -= P_i X_jc
            for c in range(j + 1):
                Xjc = D[j] if c == j else D[j] @ Bt[j, c]
                X[j, c] = Xjc
                Bt[i, c] = Bt.get((i, c), np.zeros((B, B))) - Pi[i] @ Xjc
        D[s] = Ds
        Lout[s, s] = Lss
    j = nb - 1
    for c in range(j + 1):
        X[j, c] = D[j] if c == j else D[j] @ Bt[j, c]
    M = nb * B
    L = np.zeros((M, M)); Xi = np.zeros((M, M))
    for (i, l), t in Lout.items(): L[i * B:(i + 1) * B, l * B:(l + 1) * B] = t
    for (i, l), t in X.items(): Xi[i * B:(i + 1) * B, l * B:(l + 1) * B] = t
    return L, Xi


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    for nb in (2, 3, 4, 6, 9):
        M = 64 * nb
        Z = rng.standard_normal((M, 4))
        d2 = ((Z[:, None, :] - Z[None, :, :]) ** 2).sum(-1)
        Kuu = np.exp(-0.5 * d2 / 1.5 ** 2) + 1e-3 * np.eye(M)
        L, Xi = simulate(Kuu, nb)
        Lr = np.linalg.cholesky(Kuu)
        print(nb, np.abs(L - Lr).max() / np.abs(Lr).max(), np.abs(Xi - np.linalg.inv(Lr)).max() / np.abs(np.linalg.inv(Lr)).max())
