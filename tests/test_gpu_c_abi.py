"""The C-ABI on its own: tests/c_abi/elbo_c (a host program linked against
libmgp_hip.so only -- no torch, no Python; built by __graft_entry__.build()) runs one
SMGP ELBO through the split-f16 chain of INTEGRATION.md §2 (mgp_kuu_potrf_trtri,
mgp_rbf_kuf_f16, mgp_split_upper_f16, mgp_trsm_stats_f16, mgp_split_lower_f16,
mgp_expert_conditional_f16, mgp_gauss_kl_white, mgp_elbo_terms, mgp_elbo_combine) on
hipMalloc'd buffers, with explicit noise; its ELBO against the float64 oracle (1e-4,
the north_star gate) and against the Python host's _build_likelihood on the same inputs.
The same program with --front runs the SURVEY §8(b) names only."""
import os
import subprocess

import numpy as np
import pytest
import torch

from oracle import cpu_ref as R
from tests.helpers import build_model, dev_noise

pytestmark = pytest.mark.gpu

BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_abi", "elbo_c")


def _write_problem(path, X, Y, p, z, u):
    N, D = X.shape
    M, K = p.pred["q_mu"].shape
    S = z.shape[0]
    f32 = lambda a: np.ascontiguousarray(np.asarray(a, np.float32))
    with open(path, "wb") as f:
        f.write(np.array([N, M, K, D, S], np.int64).tobytes())
        f.write(np.array([p.num_data], np.float64).tobytes())
        f.write(f32(X).tobytes())
        f.write(f32(Y.reshape(-1)).tobytes())
        for L in (p.pred, p.assign):
            f.write(f32(L["Z"]).tobytes())
            f.write(f32([L["variance"]]).tobytes())
            f.write(f32([np.ravel(L["lengthscales"])[0]]).tobytes())
            f.write(f32(L["q_mu"]).tobytes())
            f.write(f32(L["q_sqrt"]).tobytes())
        f.write(f32(np.ravel(p.lik_variance)).tobytes())
        f.write(f32(z).tobytes())
        f.write(f32(u).tobytes())


@pytest.mark.parametrize("N,M,K,D,ls,S", [(2000, 64, 3, 2, 0.8, 5), (4099, 130, 4, 3, 1.0, 9),
                                          (65536, 1024, 8, 8, 1.0, 25)])   # BASELINE config 3 in full
def test_elbo_through_the_c_abi_alone(device, tmp_path, N, M, K, D, ls, S):
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} is missing: run __graft_entry__.build() (it builds the C-ABI host program)")
    X, Y, p = R.synthetic_problem(N, M, K, D, ls, state="perturbed", S=S)
    z, u = R.explicit_noise(S, N, K, seed=5)
    prob = tmp_path / "problem.bin"
    _write_problem(prob, X, Y, p, z, u)
    r = subprocess.run([BIN, str(prob)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = dict(l.split(" ", 1) for l in r.stdout.strip().splitlines())
    assert lines["info"].split() == ["0", "0"]
    elbo_c = float(lines["elbo"])
    ref = R.smgp_elbo(X, Y, p, z, u)
    model = build_model(p, device, seed=7)
    from modulatedgps_amd import config
    old = config.expert_format()
    config.set_expert_format("f16")
    try:
        e_py = float(model._build_likelihood(torch.as_tensor(X, dtype=torch.float32, device=device), Y,
                                             noise=dev_noise(z, u, device)).cpu())
    finally:
        config.set_expert_format(old)
    print(f"C-ABI {elbo_c:.9g}  python {e_py:.9g}  oracle {ref:.9g}")
    assert elbo_c == pytest.approx(ref, rel=1e-4)
    assert elbo_c == pytest.approx(e_py, rel=1e-5)
    # both layers' K4 / K5 through the batch entries: the same bits
    rb = subprocess.run([BIN, str(prob), "--batched"], capture_output=True, text=True, timeout=120)
    assert rb.returncode == 0, rb.stderr
    assert rb.stdout == r.stdout
    # the SURVEY §8(b) front names alone (mgp_rbf_kuu_jitter -> mgp_potrf_lower -> mgp_rbf_kuf ->
    # mgp_trsm_lln -> mgp_expert_conditional -> mgp_gauss_kl_white).  Its Kuu is float32 (the
    # front's interface) where the fused chain builds it in float64; measured (round 6): rel
    # 1.8e-5 at cond(Kuu) 1.1e7, 1.2e-6 at 7.6e6, 5.3e-8 at BASELINE config 3 (cond 4.8e2)
    rf = subprocess.run([BIN, str(prob), "--front"], capture_output=True, text=True, timeout=120)
    assert rf.returncode == 0, rf.stdout + rf.stderr
    lf = dict(l.split(" ", 1) for l in rf.stdout.strip().splitlines())
    assert lf["info"].split() == ["0", "0"]
    elbo_front = float(lf["elbo"])
    cond = max(np.linalg.cond(R.rbf_Kuu(L["Z"], L["variance"], L["lengthscales"])) for L in (p.pred, p.assign))
    print(f"front {elbo_front:.9g} (rel {abs(elbo_front - ref) / abs(ref):.2e}, cond(Kuu) {cond:.2e})")
    assert elbo_front == pytest.approx(ref, rel=1e-4)
