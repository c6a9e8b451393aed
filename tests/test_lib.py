"""CPU tests of the C-ABI boundary: libmgp_hip.so loads without a GPU and exports
every function declared in include/mgp_hip.h (no compute calls are made)."""
import os
import ctypes

import pytest

from modulatedgps_amd import _lib


def test_library_loads_and_reports_gfx950():
    lib = _lib.load()
    assert lib.mgp_version().decode().endswith("gfx950")


def test_exports_every_header_symbol():
    syms = _lib.header_symbols()
    assert len(syms) >= 18
    raw = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(raw, s)]
    assert not missing, missing


def test_binding_table_matches_header():
    assert sorted(_lib.SIGNATURES) == _lib.header_symbols()


def test_status_strings_and_argument_checks():
    lib = _lib.load()
    assert lib.mgp_status_string(0) == b"ok"
    assert b"workspace" in lib.mgp_status_string(1)
    # invalid arguments are rejected before any HIP call (safe without a GPU)
    assert lib.mgp_rbf_kuf(None, 1, None, 1, 10, 10, 1, None, None, 1, None, 12, None) == -1
    assert lib.mgp_trsm_stats(None, 0, None, 0, 4, 4, None, 0, 1, None, 0, None, 0, None) == -1
    # per matrix float64 W, B [Mp][Mp] + D [nb][64][64]
    assert lib.mgp_chol_workspace_bytes(1024, 2) == 2 * (2 * 1024 * 1024 + 16 * 64 * 64) * 8
    assert lib.mgp_stats_tiles(1024) in (8, 16)   # 128- or 64-row tiles


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(_lib.MGPLibraryError):
        _lib.load()


def test_binding_arities_match_header():
    """Each ctypes prototype has as many arguments as the header declaration."""
    import re
    text = re.sub(r"/\*.*?\*/", "", open(_lib.HEADER_PATH).read(), flags=re.S)
    for name, (_, args) in _lib.SIGNATURES.items():
        m = re.search(r"\b" + name + r"\s*\(([^;]*?)\)\s*;", text, re.S)
        assert m, name
        decl = m.group(1).strip()
        n = 0 if decl in ("", "void") else decl.count(",") + 1
        assert n == len(args), (name, n, len(args))


def test_jitter_argument_is_validated():
    """The reparameterisation jitter (default_jitter(), utils.py:26-27) is an ABI
    argument of K6 and the sampler; a negative value is rejected before any HIP call."""
    lib = _lib.load()
    c = ctypes.c_void_p(8)
    rc = lib.mgp_elbo_terms(c, c, c, c, 4, c, c, 4, 2, 3, 0.01, -1.0, None, None, 0, 0, c, c, 64, None)
    assert rc == -14


def test_library_reads_no_environment():
    """the only process-global state is the lazily loaded code object --
    kernel choices follow from the entry point and its arguments, so the library
    imports no getenv (round 4 removed its per-call variant switches)."""
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"getenv\x00" not in data


def test_integration_lists_every_entry():
    """INTEGRATION.md §2a names every C-ABI entry of include/mgp_hip.h (with the
    reference call site it replaces)."""
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "INTEGRATION.md")).read()
    missing = [s for s in _lib.header_symbols() if f"`{s}`" not in text]
    assert not missing, missing


def test_batch_entries_reject_out_of_range_batch():
    """The layer-batch entries take batch in [1, 2] and reject anything else with a
    code of their own (documented in mgp_hip.h) before any HIP call."""
    lib = _lib.load()
    p = (ctypes.c_void_p * 3)(8, 8, 8)
    assert lib.mgp_split_upper_f16_bounded_batch(3, ctypes.c_void_p(8), 64, 4096, 64, p, 1 << 20, None) == -9
    assert lib.mgp_split_upper_f16_bounded_batch(0, ctypes.c_void_p(8), 64, 4096, 64, p, 1 << 20, None) == -9
    assert lib.mgp_split_upper_f16_bounded_batch(1, None, 64, 4096, 64, p, 1 << 20, None) == -2
    for bad in (0, 3):
        assert lib.mgp_qsqrt_images_kl_f16_batch(bad, p, 8, p, 64, 4096, 64, 8, p, 1 << 24, p, p, 1 << 20,
                                                 None) == -1
    assert lib.mgp_qsqrt_images_kl_f16_batch(2, None, 8, p, 64, 4096, 64, 8, p, 1 << 24, p, p, 1 << 20, None) == -2
    assert lib.mgp_qsqrt_images_kl_f16_batch(2, p, 8, p, 64, 4096, 64, 8, p, 16, p, p, 1 << 20, None) == -10


def test_tail_backward_batch_entries_check_arguments():
    """mgp_chol_backward_batch / mgp_rbf_backward_batch: batch in [1, 8], per-layer NULL
    pointers and sizes rejected with the codes documented in mgp_hip.h, a short
    workspace with MGP_ERR_WORKSPACE -- all before any HIP call."""
    lib = _lib.load()
    c = ctypes.c_void_p(8)
    p = (ctypes.c_void_p * 2)(8, 8)
    z = (ctypes.c_void_p * 2)(8, None)
    for bad in (0, 9):
        assert lib.mgp_chol_backward_batch(bad, p, 64, p, 64, p, 64, 64, p, 64, c, 1 << 30, None) == -1
        assert lib.mgp_rbf_backward_batch(bad, c, 8, 100, p, 8, 64, 8, p, p, 1, p, 100, p, 64, 1, p, 8, p, p,
                                          c, 1 << 30, None) == -1
    assert lib.mgp_chol_backward_batch(2, z, 64, p, 64, p, 64, 64, p, 64, c, 1 << 30, None) == -2
    assert lib.mgp_chol_backward_batch(2, p, 64, p, 64, z, 64, 64, p, 64, c, 1 << 30, None) == -6
    assert lib.mgp_chol_backward_batch(2, p, 64, p, 64, p, 64, -1, p, 64, c, 1 << 30, None) == -8
    assert lib.mgp_chol_backward_batch(2, p, 64, p, 64, p, 64, 64, p, 32, c, 1 << 30, None) == -10
    ws = lib.mgp_chol_backward_workspace_bytes(64)
    assert lib.mgp_chol_backward_batch(2, p, 64, p, 64, p, 64, 64, p, 64, c, 2 * ws - 1, None) == 1
    args = lambda **kw: [kw.get(k, v) for k, v in (
        ("batch", 2), ("X", c), ("ldx", 8), ("N", 100), ("Z", p), ("ldz", 8), ("M", 64), ("D", 8), ("var", p),
        ("ls", p), ("n_ls", 1), ("gKuf", p), ("ldgf", 100), ("gKuu", p), ("ldgu", 64), ("acc", 1), ("gZ", p),
        ("ldgz", 8), ("g_var", p), ("g_ls", p), ("ws", c), ("wsb", 1 << 30), ("s", None))]
    assert lib.mgp_rbf_backward_batch(*args(X=None)) == -2
    assert lib.mgp_rbf_backward_batch(*args(D=33, ldx=64, ldz=64, ldgz=64)) == 3
    assert lib.mgp_rbf_backward_batch(*args(n_ls=3)) == -11
    assert lib.mgp_rbf_backward_batch(*args(gKuu=z)) == -14
    assert lib.mgp_rbf_backward_batch(*args(g_ls=z)) == -19
    assert lib.mgp_rbf_backward_batch(*args(acc=3)) == -20 and lib.mgp_rbf_backward_batch(*args(acc=-1)) == -20
    wb = lib.mgp_rbf_backward_batch_workspace_bytes(100, 64, 8)
    assert lib.mgp_rbf_backward_batch(*args(wsb=2 * wb - 1)) == 1


def test_adam_step_set_checks_arguments():
    """mgp_adam_step_set: n in [1, 16], NULL arrays / entries and bad sizes rejected
    with the codes of mgp_hip.h before any HIP call; all-empty blocks are a no-op."""
    lib = _lib.load()
    P, I64, I32 = ctypes.c_void_p * 2, ctypes.c_int64 * 2, ctypes.c_int32 * 2
    p, z = P(8, 8), P(8, None)
    one, i32 = I64(4, 4), I32(0, 1)
    call = lambda n=2, theta=p, u=p, g=p, m1=p, rows=one, cols=one, ld=one, t=1: lib.mgp_adam_step_set(
        n, theta, u, g, i32, one, m1, p, rows, cols, ld, 1e-3, 0.9, 0.999, 1e-7, t, -1.0, None)
    assert call(n=0) == -1 and call(n=17) == -1
    assert call(theta=z) == -2
    assert call(theta=z, rows=I64(0, 0)) == 0   # an empty block's pointers are not used
    assert call(g=z) == -4
    assert call(m1=z) == -7
    assert call(rows=I64(4, -1)) == -9
    assert call(ld=I64(4, 3)) == -11
    assert call(t=0) == -16
    assert call(rows=I64(0, 0)) == 0   # nothing to update: no launch


def test_conditional_backward_prep_entries_check_arguments():
    """mgp_conditional_backward_prep_f16c / _f16c_prepped: NULL pointers, bad sizes and a
    short prep buffer rejected with the codes of mgp_hip.h before any HIP call."""
    lib = _lib.load()
    c = ctypes.c_void_p(256)
    M, K, N = 64, 3, 100
    pb = lib.mgp_conditional_backward_prep_bytes(M, K)
    assert pb >= lib.mgp_x6_lower_bytes(M, K) + K * M * M * 4
    prep = lambda q=c, ldqs=M, sq=M * M, m=M, k=K, lb=c, out=c, nb=pb: lib.mgp_conditional_backward_prep_f16c(
        q, ldqs, sq, m, k, lb, out, nb, None)
    assert prep(q=None) == -1 and prep(ldqs=M - 1) == -2 and prep(sq=M) == -3
    assert prep(m=0) == -4 and prep(k=0) == -5 and prep(k=17) == 3
    assert prep(lb=None) == -6 and prep(out=None) == -7 and prep(nb=pb - 1) == 1
    assert prep(out=ctypes.c_void_p(264)) == 2
    wsb = lib.mgp_conditional_backward_workspace_bytes(M, N, K)
    cb = lambda cfr=c, pr=c, nb=pb: lib.mgp_conditional_backward_f16c_prepped(
        c, 1 << 30, c, 128, c, M, M * M, c, K, c, M, c, c, 128, M, N, K, c, K, c, M, M * M, c, 128, c, M, c, c, wsb,
        cfr, 1 << 30, c, c, pr, nb, None, None)
    assert cb(cfr=None) == -30 and cb(pr=None) == -33 and cb(nb=pb - 1) == -34
