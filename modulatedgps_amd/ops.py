"""Torch-tensor wrappers over the libmgp_hip C-ABI (device memory + streams only).

PyTorch is used here as plumbing: it allocates device buffers and supplies the
current HIP stream.  Every arithmetic op runs in a hand-written gfx950 kernel
of libmgp_hip.so; nothing here computes on the CPU or with torch kernels.

Layout conventions (see include/mgp_hip.h): float32, row-major, leading
dimensions padded to a multiple of 4 elements so rows can be read as float4.
``padded(rows, cols)`` returns such a view; the expert-major conditional
outputs are [K][N] views.
"""
import ctypes
import torch

from . import _lib
from .config import default_jitter

F32 = torch.float32


def _round4(x):
    return (int(x) + 3) // 4 * 4


def _stream():
    return ctypes_stream(torch.cuda.current_stream())


def ctypes_stream(s):
    return s.cuda_stream


def padded(rows, cols, device, batch=None, dtype=F32, zero=False):
    """[batch?][rows][cols] view over storage whose rows are padded to a multiple of 4."""
    ld = _round4(max(cols, 1))
    shape = (rows, ld) if batch is None else (batch, rows, ld)
    fn = torch.zeros if zero else torch.empty
    buf = fn(shape, dtype=dtype, device=device)
    return buf[..., :cols]


def as_padded(t, device=None, dtype=F32):
    """Copy a 2-D/3-D tensor (or array) into padded storage (unless it already is)."""
    t = torch.as_tensor(t)
    device = device or t.device
    if (t.device == torch.device(device) and t.dtype == dtype and t.stride(-1) == 1
            and t.stride(-2) % 4 == 0 and t.data_ptr() % 16 == 0
            and (t.dim() == 2 or t.stride(0) % 4 == 0)):
        return t
    out = padded(t.shape[-2], t.shape[-1], device, batch=t.shape[0] if t.dim() == 3 else None,
                 dtype=dtype)
    out.copy_(t.to(device=device, dtype=dtype))
    return out


def _ld(t):
    if t.stride(-1) != 1:
        raise ValueError("innermost dimension must be contiguous")
    return t.stride(-2) if t.dim() >= 2 else t.shape[-1]


def _check(t, name, ndim=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != F32:
        raise TypeError(f"{name} must be float32, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name} must be {ndim}-D, got shape {tuple(t.shape)}")


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


# --------------------------------------------------------------------------- K1 / K2
def rbf_kuf(X, Z, variance, lengthscales, out=None):
    """Kuf = K(Z, X) [M, N] (models.py:139)."""
    _check(X, "X", 2), _check(Z, "Z", 2), _check(variance, "variance"), _check(lengthscales, "lengthscales")
    N, D = X.shape
    M = Z.shape[0]
    if Z.shape[1] != D:
        raise ValueError("X and Z must have the same number of columns")
    if out is None:
        out = padded(M, N, X.device)
    _lib.call("mgp_rbf_kuf", X.data_ptr(), _ld(X), Z.data_ptr(), _ld(Z), N, M, D,
              variance.data_ptr(), lengthscales.data_ptr(), lengthscales.numel(), out.data_ptr(),
              _ld(out), _stream())
    return out


def rbf_kuu(Z, variance, lengthscales, jitter, out=None):
    """Kuu = K(Z, Z) + jitter I [M, M] (models.py:135)."""
    _check(Z, "Z", 2)
    M, D = Z.shape
    if out is None:
        out = padded(M, M, Z.device)
    _lib.call("mgp_rbf_kuu", Z.data_ptr(), _ld(Z), M, D, variance.data_ptr(), lengthscales.data_ptr(),
              lengthscales.numel(), float(jitter), out.data_ptr(), _ld(out), _stream())
    return out


# --------------------------------------------------------------------------- K3
def potrf_trtri(A, L=None, LinvT=None, info=None, workspace=None):
    """Batched Cholesky + inverse of A [B, M, M] (lower part read).
    Returns L [B,M,M], LinvT [B,M,M] and info int32 [B] (device; 0 = success)."""
    _check(A, "A", 3)
    Bt, M, _ = A.shape
    dev = A.device
    if L is None:
        L = padded(M, M, dev, batch=Bt)
    if LinvT is None:
        LinvT = padded(M, M, dev, batch=Bt)
    if info is None:
        info = torch.empty(Bt, dtype=torch.int32, device=dev)
    nbytes = _lib.load().mgp_chol_workspace_bytes(M, Bt)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    if L.stride(0) != LinvT.stride(0) or _ld(L) != _ld(LinvT):
        raise ValueError("L and LinvT must share a layout")
    _lib.call("mgp_potrf_trtri", A.data_ptr(), _ld(A), A.stride(0), M, Bt, L.data_ptr(),
              LinvT.data_ptr(), _ld(L), L.stride(0), info.data_ptr(), workspace.data_ptr(),
              workspace.numel(), _stream())
    return L, LinvT, info


def kuu_potrf_trtri(Zs, variances, lengthscales, jitter, LinvT=None, L=None, info=None,
                    workspace=None, want_L=False, prep_event=None, tfr_bound_images=None, kuf=None):
    """Kuu (float64, from Z) + Cholesky + inverse for a batch of layers sharing M, D.
    Zs / variances / lengthscales: lists of device tensors.  Returns L (or None),
    LinvT [B, M, M] and info int32 [B].  prep_event: a torch.cuda.Event (already
    created) recorded once Kuu is built (mgp_kuu_potrf_trtri_ev).
    tfr_bound_images: per layer, the L^-T split-f16 image buffer whose trailer
    receives max |LinvT| (mgp_kuu_potrf_trtri_ex; then split_upper_x6(...,
    bounded=True) skips its reduction).
    kuf: (X [N, D], [image per layer], fmt "f16" | "x6"): the factorisation's step
    launches also write each layer's Kuf image K(Z_b, X), bit-identical to
    rbf_kuf_x6(X, Z_b, ..., fmt=fmt) (mgp_kuu_potrf_trtri_kuf)."""
    import ctypes
    Bt = len(Zs)
    M, D = Zs[0].shape
    ldz = _ld(Zs[0])
    for Z in Zs:
        _check(Z, "Z", 2)
        if tuple(Z.shape) != (M, D) or _ld(Z) != ldz:
            raise ValueError("all Z must share shape and leading dimension")
    dev = Zs[0].device
    if LinvT is None:
        LinvT = padded(M, M, dev, batch=Bt)
    if want_L and L is None:
        L = padded(M, M, dev, batch=Bt)
    if info is None:
        info = torch.empty(Bt, dtype=torch.int32, device=dev)
    nbytes = _lib.load().mgp_chol_workspace_bytes(M, Bt)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    P = ctypes.c_void_p * Bt
    zp = P(*[z.data_ptr() for z in Zs])
    vp = P(*[v.data_ptr() for v in variances])
    lp = P(*[l.data_ptr() for l in lengthscales])
    nl = (ctypes.c_int32 * Bt)(*[l.numel() for l in lengthscales])
    if kuf is not None:
        lib = _lib.load()
        X, imgs, fmt = kuf
        _check(X, "X", 2)
        if X.shape[1] != D or len(imgs) != Bt:
            raise ValueError("kuf: X must have Z's D columns and one image per layer")
        kb = lib.mgp_x6_cols_bytes(M, X.shape[0])
        if min(t.numel() for t in imgs) < kb:
            raise ValueError("kuf: an image buffer is smaller than mgp_x6_cols_bytes(M, N)")
        bp = None
        if tfr_bound_images is not None:
            bp = P(*[lib.mgp_x6_bound_ptr(t.data_ptr(), M, 0, 1) for t in tfr_bound_images])
        _lib.call("mgp_kuu_potrf_trtri_kuf", zp, ldz, M, D, vp, lp, nl, float(jitter), Bt,
                  L.data_ptr() if L is not None else None, LinvT.data_ptr(), _ld(LinvT),
                  LinvT.stride(0), info.data_ptr(), workspace.data_ptr(), workspace.numel(),
                  prep_event.cuda_event if prep_event is not None else None, bp,
                  X.data_ptr(), _ld(X), X.shape[0], P(*[t.data_ptr() for t in imgs]),
                  min(t.numel() for t in imgs), {"x6": 0, "f16": 1}[fmt], _stream())
    elif tfr_bound_images is not None:
        lib = _lib.load()
        bp = P(*[lib.mgp_x6_bound_ptr(t.data_ptr(), M, 0, 1) for t in tfr_bound_images])
        _lib.call("mgp_kuu_potrf_trtri_ex", zp, ldz, M, D, vp, lp, nl, float(jitter), Bt,
                  L.data_ptr() if L is not None else None, LinvT.data_ptr(), _ld(LinvT),
                  LinvT.stride(0), info.data_ptr(), workspace.data_ptr(), workspace.numel(),
                  prep_event.cuda_event if prep_event is not None else None, bp, _stream())
    elif prep_event is not None:
        _lib.call("mgp_kuu_potrf_trtri_ev", zp, ldz, M, D, vp, lp, nl, float(jitter), Bt,
                  L.data_ptr() if L is not None else None, LinvT.data_ptr(), _ld(LinvT),
                  LinvT.stride(0), info.data_ptr(), workspace.data_ptr(), workspace.numel(),
                  prep_event.cuda_event, _stream())
    else:
        _lib.call("mgp_kuu_potrf_trtri", zp, ldz, M, D, vp, lp, nl, float(jitter), Bt,
                  L.data_ptr() if L is not None else None, LinvT.data_ptr(), _ld(LinvT),
                  LinvT.stride(0), info.data_ptr(), workspace.data_ptr(), workspace.numel(), _stream())
    return L, LinvT, info


def check_info(info):
    """Raise MGPLinAlgError if any factorisation reported a bad pivot (host sync)."""
    bad = info.cpu()
    if bool((bad != 0).any()):
        raise _lib.MGPLinAlgError("mgp_potrf_trtri", int(bad.max()),
                                  "Cholesky decomposition was not successful: the input might "
                                  "not be valid (non-positive pivot at column %s)" % bad.tolist())


# --------------------------------------------------------------------------- K4 / K5
def stats_tiles(M):
    return _lib.load().mgp_stats_tiles(M)


def trsm_stats(LinvT, Kuf, q_mu, A=None, stats=None):
    """A = L^-1 Kuf and per-row-tile column stats [T, K+1, N]."""
    _check(LinvT, "LinvT", 2), _check(Kuf, "Kuf", 2), _check(q_mu, "q_mu", 2)
    M, N = Kuf.shape
    K = q_mu.shape[1]
    dev = Kuf.device
    if A is None:
        A = padded(M, N, dev)
    if stats is None:
        T = stats_tiles(M)
        stats = padded(T * (K + 1), N, dev).unflatten(0, (T, K + 1))
    _lib.call("mgp_trsm_stats", LinvT.data_ptr(), _ld(LinvT), Kuf.data_ptr(), _ld(Kuf), M, N,
              q_mu.data_ptr(), _ld(q_mu), K, A.data_ptr(), _ld(A), stats.data_ptr(), _ld(stats),
              _stream())
    return A, stats


def rbf_kuf_x6(X, Z, variance, lengthscales, out=None, fmt="x6"):
    """K1 writing the split-bf16 image of Kuf = K(Z, X) (uint8 device tensor);
    fmt "f16": the split-f16 image (mgp_rbf_kuf_f16) for trsm_stats_x6(..., in_fmt="f16")."""
    _check(X, "X", 2), _check(Z, "Z", 2)
    N, D = X.shape
    M = Z.shape[0]
    nbytes = _lib.load().mgp_x6_cols_bytes(M, N)
    if out is None or out.numel() < nbytes:
        out = _ws(nbytes, X.device)
    _lib.call("mgp_rbf_kuf_" + _fmt(fmt), X.data_ptr(), _ld(X), Z.data_ptr(), _ld(Z), N, M, D, variance.data_ptr(),
              lengthscales.data_ptr(), lengthscales.numel(), out.data_ptr(), out.numel(), _stream())
    return out


def split_upper_x6(LinvT, out=None, fmt="x6", bounded=False):
    """Split-bf16 image of (L^-1)^T [M, M] (upper triangle) as K4's T operand
    (fmt "f16": the split-f16 image, mgp_split_upper_f16; bounded: `out`'s trailer
    already holds max |LinvT| from kuu_potrf_trtri(..., tfr_bound_images=...),
    mgp_split_upper_f16_bounded)."""
    _check(LinvT, "LinvT", 2)
    M = LinvT.shape[0]
    nbytes = _lib.load().mgp_x6_lower_bytes(M, 1)
    if bounded and (fmt != "f16" or out is None):
        raise ValueError("bounded splits are split-f16 into the image that received the bound")
    if out is None or out.numel() < nbytes:
        out = _ws(nbytes, LinvT.device)
    name = "mgp_split_upper_f16_bounded" if bounded else "mgp_split_upper_" + _fmt(fmt)
    _lib.call(name, LinvT.data_ptr(), _ld(LinvT), M, out.data_ptr(), out.numel(), _stream())
    return out


def split_upper_f16_bounded_batch(LinvT, outs):
    """split_upper_x6(LinvT[b], out=outs[b], fmt="f16", bounded=True) for every matrix of
    LinvT [B, M, M] (B = len(outs) <= 2) in one launch (mgp_split_upper_f16_bounded_batch)."""
    _check(LinvT, "LinvT", 3)
    n, M = len(outs), LinvT.shape[1]
    if LinvT.shape[0] < n:
        raise ValueError("one LinvT matrix per image")
    arr = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    _lib.call("mgp_split_upper_f16_bounded_batch", n, LinvT.data_ptr(), _ld(LinvT), LinvT.stride(0), M, arr,
              min(o.numel() for o in outs), _stream())
    return list(outs)


def trsm_stats_x6(Tfr, Kfr, q_mu, M, N, Afr=None, stats=None, A=None, f16_variance=None, in_fmt="x6", cross=None):
    """K4 on images: A's image (for expert_conditional_x6) and the stats [T, K+1, N];
    also the f32 A when a buffer `A` [M, N] is given (training).  f16_variance
    (the layer's kernel variance): A's image is split-f16 instead
    (mgp_trsm_stats_x6_f16, for expert_conditional_x6(..., fmt="f16")).
    in_fmt "f16": Tfr and Kfr are split-f16 images (split_upper_x6 / rbf_kuf_x6 with
    fmt "f16"; mgp_trsm_stats_f16, needs f16_variance).
    cross "f8" (default: config.expert_cross()) with split-f16 inputs: A's image also
    carries the e4m3 cross-term plane of expert_conditional_x6(..., cross="f8")
    (mgp_trsm_stats_f16x8)."""
    _check(q_mu, "q_mu", 2)
    K = q_mu.shape[1]
    dev = q_mu.device
    nbytes = _lib.load().mgp_x6_cols_bytes(M, N)
    if Afr is None or Afr.numel() < nbytes:
        Afr = _ws(nbytes, dev)
    if stats is None:
        T = stats_tiles(M)
        stats = padded(T * (K + 1), N, dev).unflatten(0, (T, K + 1))
    if f16_variance is not None:
        if _fmt(in_fmt) == "x6":
            if A is not None:
                raise ValueError("the split-bf16 -> split-f16 K4 does not write the f32 A")
            _lib.call("mgp_trsm_stats_x6_f16", Tfr.data_ptr(), Tfr.numel(), Kfr.data_ptr(), Kfr.numel(), M, N,
                      q_mu.data_ptr(), _ld(q_mu), K, f16_variance.data_ptr(), Afr.data_ptr(), Afr.numel(),
                      stats.data_ptr(), _ld(stats), _stream())
        else:
            from .config import expert_cross
            entry = "mgp_trsm_stats_f16x8" if (cross or expert_cross()) == "f8" else "mgp_trsm_stats_f16"
            _lib.call(entry, Tfr.data_ptr(), Tfr.numel(), Kfr.data_ptr(), Kfr.numel(), M, N,
                      q_mu.data_ptr(), _ld(q_mu), K, f16_variance.data_ptr(), Afr.data_ptr(), Afr.numel(),
                      stats.data_ptr(), _ld(stats), A.data_ptr() if A is not None else None,
                      _ld(A) if A is not None else N, _stream())
        return Afr, stats
    if _fmt(in_fmt) != "x6":
        raise ValueError("split-f16 K4 inputs need the split-f16 output (f16_variance)")
    _lib.call("mgp_trsm_stats_x6", Tfr.data_ptr(), Tfr.numel(), Kfr.data_ptr(), Kfr.numel(), M, N,
              q_mu.data_ptr(), _ld(q_mu), K, Afr.data_ptr(), Afr.numel(), stats.data_ptr(), _ld(stats),
              A.data_ptr() if A is not None else None, _ld(A) if A is not None else N, _stream())
    return Afr, stats


def trsm_stats_f16_batch(Tfrs, Kfrs, q_mus, M, N, Afrs, statss, variances, As=None):
    """K4 of several layers (1 or 2, equal M, N, K) in one launch (mgp_trsm_stats_f16_batch):
    trsm_stats_x6(Tfr, Kfr, q_mu, M, N, Afr=Afr, stats=stats, A=A, f16_variance=variance,
    in_fmt="f16", cross="f16") for each layer, bit-identical.  Afrs / statss: the output
    buffers (required); As: f32 A buffers or None."""
    n = len(Tfrs)
    for seq in (Kfrs, q_mus, Afrs, statss, variances) + ((As,) if As is not None else ()):
        if len(seq) != n:
            raise ValueError("one entry per layer in every operand list")
    K = q_mus[0].shape[1]
    ldq, lds = _ld(q_mus[0]), _ld(statss[0])
    for q, st in zip(q_mus, statss):
        _check(q, "q_mu", 2)
        if q.shape[1] != K or _ld(q) != ldq or _ld(st) != lds:
            raise ValueError("the layers' q_mu / stats must share K and leading dimensions")
    lda = N
    if As is not None:
        lda = _ld(As[0])
        if any(_ld(a) != lda for a in As):
            raise ValueError("the f32 A buffers must share a leading dimension")

    def arr(ts):
        return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    _lib.call("mgp_trsm_stats_f16_batch", n, arr(Tfrs), min(t.numel() for t in Tfrs), arr(Kfrs),
              min(t.numel() for t in Kfrs), M, N, arr(q_mus), ldq, K, arr(variances), arr(Afrs),
              min(t.numel() for t in Afrs), arr(statss), lds, arr(As) if As is not None else None, lda, _stream())
    return list(zip(Afrs, statss))


def expert_workspace_bytes(M, N, K):
    return max(int(_lib.load().mgp_expert_workspace_bytes(M, N, K)), 16)


def expert_x6_workspace_bytes(M, N, K):
    return max(int(_lib.load().mgp_expert_x6_workspace_bytes(M, N, K)), 16)


def x6_cols_bytes(M, N):
    return int(_lib.load().mgp_x6_cols_bytes(M, N))


def x6_lower_bytes(M, K):
    return int(_lib.load().mgp_x6_lower_bytes(M, K))


def expert_conditional(A, q_sqrt, stats, variance, fmean=None, fvar=None, workspace=None):
    """fmean, fvar [K, N] of the whitened K-expert conditional."""
    _check(A, "A", 2), _check(q_sqrt, "q_sqrt", 3), _check(stats, "stats", 3)
    M, N = A.shape
    K = q_sqrt.shape[0]
    dev = A.device
    if fmean is None:
        fmean = padded(K, N, dev)
    if fvar is None:
        fvar = padded(K, N, dev)
    if _ld(fmean) != _ld(fvar):
        raise ValueError("fmean and fvar must share a leading dimension")
    nbytes = _lib.load().mgp_expert_workspace_bytes(M, N, K)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    _lib.call("mgp_expert_conditional_f32", A.data_ptr(), _ld(A), q_sqrt.data_ptr(), _ld(q_sqrt),
              q_sqrt.stride(0), stats.data_ptr(), _ld(stats), variance.data_ptr(), M, N, K,
              fmean.data_ptr(), fvar.data_ptr(), _ld(fmean), workspace.data_ptr(),
              workspace.numel(), _stream())
    return fmean, fvar


# ------------------------------------------------------------ K5, split-bf16 (x6)
def _fmt(fmt):
    if fmt not in ("x6", "f16"):
        raise ValueError("image format must be 'x6' (split-bf16) or 'f16' (split-f16)")
    return fmt


def split_lower_x6(q_sqrt, out=None, fmt="x6"):
    """Fragment image (uint8 device tensor) of L_k = tril(q_sqrt[k]) for the split-bf16
    K5 (fmt "f16": the split-f16 image, mgp_split_lower_f16)."""
    _check(q_sqrt, "q_sqrt", 3)
    K, M = q_sqrt.shape[0], q_sqrt.shape[1]
    nbytes = _lib.load().mgp_x6_lower_bytes(M, K)
    if out is None or out.numel() < nbytes:
        out = _ws(nbytes, q_sqrt.device)
    _lib.call("mgp_split_lower_" + _fmt(fmt), q_sqrt.data_ptr(), _ld(q_sqrt), q_sqrt.stride(0), M, K,
              out.data_ptr(), out.numel(), _stream())
    return out


def qsqrt_images_kl_f16_batch(q_mus, q_sqrts, Lfrs, kl_outs, workspace=None):
    """Both layers' split-f16 tril(q_sqrt) images (split_lower_x6(q_sqrt, fmt="f16")) and
    whitened KL terms (gauss_kl_white(q_mu, q_sqrt), float64 [1] each) in three launches
    (mgp_qsqrt_images_kl_f16_batch; bit-identical).  Layers share q_mu / q_sqrt shapes."""
    import ctypes
    n = len(q_mus)
    q_sqrts = [as_padded(t) for t in q_sqrts]   # float4 rows (no copy for the layers' storage)
    M, K = q_mus[0].shape
    for qm, qs, lf, kl in zip(q_mus, q_sqrts, Lfrs, kl_outs):
        _check(qm, "q_mu", 2), _check(qs, "q_sqrt", 3)
        if (tuple(qm.shape) != (M, K) or tuple(qs.shape) != (K, M, M) or _ld(qm) != _ld(q_mus[0])
                or _ld(qs) != _ld(q_sqrts[0]) or qs.stride(0) != q_sqrts[0].stride(0)):
            raise ValueError("every layer's q_mu [M, K] / q_sqrt [K, M, M] must share shape and strides")
        if kl.dtype != torch.float64 or kl.numel() < 1:
            raise ValueError("kl_out: float64 tensors of at least one element")
    lib = _lib.load()
    nbytes = lib.mgp_qsqrt_workspace_bytes(M, K) * n
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, q_mus[0].device)
    P = ctypes.c_void_p * n
    _lib.call("mgp_qsqrt_images_kl_f16_batch", n, P(*[t.data_ptr() for t in q_mus]), _ld(q_mus[0]),
              P(*[t.data_ptr() for t in q_sqrts]), _ld(q_sqrts[0]), q_sqrts[0].stride(0), M, K,
              P(*[t.data_ptr() for t in Lfrs]), min(t.numel() for t in Lfrs), P(*[t.data_ptr() for t in kl_outs]),
              workspace.data_ptr(), workspace.numel(), _stream())
    return Lfrs, kl_outs


def split_cols_x6(A, out=None, fmt="x6"):
    """Fragment image (uint8 device tensor) of A [M, N] for the split-bf16 K5
    (fmt "f16": the split-f16 image, mgp_split_cols_f16)."""
    _check(A, "A", 2)
    M, N = A.shape
    nbytes = _lib.load().mgp_x6_cols_bytes(M, N)
    if out is None or out.numel() < nbytes:
        out = _ws(nbytes, A.device)
    _lib.call("mgp_split_cols_" + _fmt(fmt), A.data_ptr(), _ld(A), M, N, out.data_ptr(), out.numel(),
              _stream())
    return out


def expert_conditional_x6(Afr, Lfr, stats, variance, M, N, K, fmean=None, fvar=None, workspace=None, planes=3,
                          fmt="x6", cross=None, c_out=None):
    """fmean, fvar [K, N] of the whitened K-expert conditional from split-bf16 images
    (planes < 3: K5 on the leading bf16 planes only, mgp_expert_conditional_planes;
    fmt "f16": from split-f16 images, mgp_expert_conditional_f16, or with cross "f8"
    (default: config.expert_cross()) mgp_expert_conditional_f16x8, the cross terms
    on the e4m3 MFMA).  c_out = (Cfr, colmax) (f16, cross "f16"; colmax from colnorm_max):
    also write C_k = L_k^T A as images for the backward (mgp_expert_conditional_f16c)."""
    _check(stats, "stats", 3)
    dev = stats.device
    if fmean is None:
        fmean = padded(K, N, dev)
    if fvar is None:
        fvar = padded(K, N, dev)
    if _ld(fmean) != _ld(fvar):
        raise ValueError("fmean and fvar must share a leading dimension")
    nbytes = _lib.load().mgp_expert_x6_workspace_bytes(M, N, K)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    if _fmt(fmt) == "f16":
        from .config import expert_cross
        entry = "mgp_expert_conditional_f16x8" if (cross or expert_cross()) == "f8" else "mgp_expert_conditional_f16"
        args = [Afr.data_ptr(), Afr.numel(), Lfr.data_ptr(), Lfr.numel(), stats.data_ptr(), _ld(stats),
                variance.data_ptr(), M, N, K, fmean.data_ptr(), fvar.data_ptr(), _ld(fmean), workspace.data_ptr(),
                workspace.numel()]
        if c_out is not None:
            if entry != "mgp_expert_conditional_f16":
                raise ValueError("c_out needs f16 cross terms")
            Cfr, colmax = c_out
            entry = "mgp_expert_conditional_f16c"
            args += [Cfr.data_ptr(), Cfr.numel(), colmax.data_ptr()]
        _lib.call(entry, *args, _stream())
    elif planes == 3:
        _lib.call("mgp_expert_conditional_x6", Afr.data_ptr(), Afr.numel(), Lfr.data_ptr(), Lfr.numel(),
                  stats.data_ptr(), _ld(stats), variance.data_ptr(), M, N, K, fmean.data_ptr(),
                  fvar.data_ptr(), _ld(fmean), workspace.data_ptr(), workspace.numel(), _stream())
    else:
        _lib.call("mgp_expert_conditional_planes", Afr.data_ptr(), Afr.numel(), Lfr.data_ptr(), Lfr.numel(),
                  stats.data_ptr(), _ld(stats), variance.data_ptr(), M, N, K, int(planes), fmean.data_ptr(),
                  fvar.data_ptr(), _ld(fmean), workspace.data_ptr(), workspace.numel(), _stream())
    return fmean, fvar


def expert_conditional_f16_batch(Afrs, Lfrs, statss, variances, M, N, K, fmeans, fvars, workspaces, c_outs=None):
    """K5 of several layers (1 or 2, equal M, N, K) in one launch
    (mgp_expert_conditional_f16_batch): expert_conditional_x6(Afr, Lfr, stats, variance, M, N, K,
    fmean=..., fvar=..., workspace=..., fmt="f16", cross="f16", c_out=...) for each layer,
    bit-identical.  Outputs and one workspace per layer are required; c_outs: a
    (Cfr, colmax) per layer (training) or None."""
    n = len(Afrs)
    lists = (Lfrs, statss, variances, fmeans, fvars, workspaces) + ((c_outs,) if c_outs is not None else ())
    if any(len(x) != n for x in lists):
        raise ValueError("one entry per layer in every operand list")
    lds, ldf = _ld(statss[0]), _ld(fmeans[0])
    if any(_ld(t) != lds for t in statss) or any(_ld(t) != ldf for t in list(fmeans) + list(fvars)):
        raise ValueError("the layers' stats / fmean / fvar must share leading dimensions")

    def arr(ts):
        return (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])
    cf = arr([c[0] for c in c_outs]) if c_outs is not None else None
    cm = arr([c[1] for c in c_outs]) if c_outs is not None else None
    cb = min(c[0].numel() for c in c_outs) if c_outs is not None else 0
    _lib.call("mgp_expert_conditional_f16_batch", n, arr(Afrs), min(t.numel() for t in Afrs), arr(Lfrs),
              min(t.numel() for t in Lfrs), arr(statss), lds, arr(variances), M, N, K, arr(fmeans), arr(fvars), ldf,
              arr(workspaces), min(t.numel() for t in workspaces), cf, cb, cm, _stream())
    return list(zip(fmeans, fvars))


def elbo_terms_backward(mu_f, var_f, mu_a, var_a, Y, lik_var, S, tau=1e-2, noise=None, seed=0,
                        n_offset=0, scale=1.0, assign_lik_var=None, G=None, workspace=None, multiclass_eps=None,
                        jitter=None):
    """Gradient of the data term: G [4, K, N] = scale * d/d(mu_f, var_f, mu_a, var_a) and the
    likelihood-variance gradients (float64 [K]; second one for SMGPModified, else None).
    multiclass_eps: MultiClass / RobustMax pred likelihood (no likelihood-variance gradient: None)."""
    jitter = default_jitter() if jitter is None else jitter
    for t, n in ((mu_f, "mu_f"), (var_f, "var_f"), (mu_a, "mu_a"), (var_a, "var_a")):
        _check(t, n, 2)
    ldf = _ld(mu_f)
    if not (_ld(var_f) == _ld(mu_a) == _ld(var_a) == ldf):
        raise ValueError("conditional outputs must share a leading dimension")
    K, N = mu_f.shape
    dev = mu_f.device
    Y = Y.reshape(-1)
    _check(Y, "Y")
    if multiclass_eps is None:
        _check(lik_var, "lik_var")
    if G is None:
        G = padded(4 * K, N, dev).unflatten(0, (4, K))
    # the kernel addresses G's 4K rows as one [4K][ldg] block: the row stride from
    # G's outer dimension (a K = 1 view's stride(1) is torch's contiguous placeholder,
    # N, not the padded row length)
    if G.dim() != 3 or tuple(G.shape) != (4, K, N) or G.stride(2) != 1 or G.stride(0) % K:
        raise ValueError("G must be a [4, K, N] view of [4K][ldg] rows")
    ldg = G.stride(0) // K
    if K > 1 and G.stride(1) != ldg:
        raise ValueError("G must be a [4, K, N] view of [4K][ldg] rows")
    glv = torch.empty(K, dtype=torch.float64, device=dev) if multiclass_eps is None else None
    glva = torch.empty(K, dtype=torch.float64, device=dev) if assign_lik_var is not None else None
    nbytes = _lib.load().mgp_elbo_backward_workspace_bytes(N, K)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    zp = up = None
    if noise is not None:
        z, u = noise
        z, u = z.contiguous(), u.contiguous()
        zp, up = z.data_ptr(), u.data_ptr()
    if multiclass_eps is not None:
        _lib.call("mgp_elbo_terms_multiclass_backward", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(),
                  var_a.data_ptr(), ldf, Y.data_ptr(), float(multiclass_eps),
                  assign_lik_var.data_ptr() if assign_lik_var is not None else None, N, K, S, float(tau),
                  float(jitter), zp, up,
                  int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), float(scale), G.data_ptr(), ldg,
                  glva.data_ptr() if glva is not None else None, workspace.data_ptr(), workspace.numel(),
                  _stream())
        return G, glv, glva
    _lib.call("mgp_elbo_terms_backward", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(),
              var_a.data_ptr(), ldf, Y.data_ptr(), lik_var.data_ptr(),
              assign_lik_var.data_ptr() if assign_lik_var is not None else None, N, K, S, float(tau),
              float(jitter), zp, up,
              int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), float(scale), G.data_ptr(), ldg,
              glv.data_ptr(), glva.data_ptr() if glva is not None else None, workspace.data_ptr(),
              workspace.numel(), _stream())
    return G, glv, glva


def rbf_backward(X, Z, variance, lengthscales, gK, symmetric=False, accumulate=False, gZ=None, g_var=None,
                 g_ls=None, workspace=None):
    """Reverse mode of K(Z, X): (gZ [M, D] float32, g_var float64 [1], g_ls float64 [n_ls])."""
    _check(X, "X", 2), _check(Z, "Z", 2), _check(gK, "gK", 2)
    N, D = X.shape
    M = Z.shape[0]
    dev = X.device
    n_ls = lengthscales.numel()
    if gZ is None:
        gZ = torch.zeros(M, D, dtype=torch.float32, device=dev)
    if g_var is None:
        g_var = torch.zeros(1, dtype=torch.float64, device=dev)
    if g_ls is None:
        g_ls = torch.zeros(n_ls, dtype=torch.float64, device=dev)
    nbytes = _lib.load().mgp_rbf_backward_workspace_bytes(N, M, D)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    _lib.call("mgp_rbf_backward", X.data_ptr(), _ld(X), Z.data_ptr(), _ld(Z), N, M, D, variance.data_ptr(),
              lengthscales.data_ptr(), n_ls, gK.data_ptr(), _ld(gK), int(symmetric), int(accumulate),
              gZ.data_ptr(), _ld(gZ), g_var.data_ptr(), g_ls.data_ptr(), workspace.data_ptr(), workspace.numel(),
              _stream())
    return gZ, g_var, g_ls


def _same_ld(ts, what):
    if any(_ld(t) != _ld(ts[0]) for t in ts):
        raise ValueError(f"every layer's {what} must share its leading dimension")
    return _ld(ts[0])


def rbf_backward_batch(X, Zs, variances, lengthscales, gKufs, gKuus, gZs, g_vars, g_lss, accumulate=True,
                       workspace=None):
    """Per layer b: rbf_backward(X, Z[b], .., gKuf[b], accumulate) then
    rbf_backward(Z[b], Z[b], .., gKuu[b], symmetric=True, accumulate=True) into
    gZ[b], g_var[b], g_ls[b], for all layers in three launches (mgp_rbf_backward_batch;
    bit-identical).  accumulate 2: gZ / g_ls overwritten, g_var added to."""
    import ctypes
    _check(X, "X", 2)
    N, D = X.shape
    n = len(Zs)
    M = Zs[0].shape[0]
    n_ls = lengthscales[0].numel()
    for z, gf, gu in zip(Zs, gKufs, gKuus):
        _check(z, "Z", 2), _check(gf, "gKuf", 2), _check(gu, "gKuu", 2)
        if tuple(z.shape) != (M, D):
            raise ValueError("every layer's Z must be [M, D]")
    if any(t.numel() != n_ls for t in lengthscales):
        raise ValueError("every layer's lengthscales must have the same size")
    lib = _lib.load()
    nbytes = lib.mgp_rbf_backward_batch_workspace_bytes(N, M, D) * n
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, X.device)
    P = ctypes.c_void_p * n
    ptrs = lambda ts: P(*[t.data_ptr() for t in ts])
    _lib.call("mgp_rbf_backward_batch", n, X.data_ptr(), _ld(X), N, ptrs(Zs), _same_ld(Zs, "Z"), M, D,
              ptrs(variances), ptrs(lengthscales), n_ls, ptrs(gKufs), _same_ld(gKufs, "gKuf"), ptrs(gKuus),
              _same_ld(gKuus, "gKuu"), int(accumulate), ptrs(gZs), _same_ld(gZs, "gZ"), ptrs(g_vars), ptrs(g_lss),
              workspace.data_ptr(), workspace.numel(), _stream())
    return gZs, g_vars, g_lss


def chol_backward_batch(Ls, LinvTs, gLs, outs=None, workspace=None):
    """chol_backward for every layer (same M) in five launches (mgp_chol_backward_batch;
    bit-identical): list of gKuu [M, M]."""
    import ctypes
    n = len(Ls)
    M = Ls[0].shape[0]
    for t in list(Ls) + list(LinvTs) + list(gLs):
        _check(t, "L / LinvT / gL", 2)
        if tuple(t.shape) != (M, M):
            raise ValueError("every layer's L, LinvT and gL must be [M, M]")
    if outs is None:
        outs = [padded(M, M, Ls[0].device) for _ in range(n)]
    nbytes = _lib.load().mgp_chol_backward_workspace_bytes(M) * n
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, Ls[0].device)
    P = ctypes.c_void_p * n
    ptrs = lambda ts: P(*[t.data_ptr() for t in ts])
    _lib.call("mgp_chol_backward_batch", n, ptrs(Ls), _same_ld(Ls, "L"), ptrs(LinvTs), _same_ld(LinvTs, "LinvT"),
              ptrs(gLs), _same_ld(gLs, "gL"), M, ptrs(outs), _same_ld(outs, "gKuu"), workspace.data_ptr(),
              workspace.numel(), _stream())
    return outs


def chol_backward(L, LinvT, gL, out=None, workspace=None):
    """gKuu [M, M] (float32, symmetric) from the gradient w.r.t. Lm = chol(Kuu)."""
    _check(L, "L", 2), _check(LinvT, "LinvT", 2), _check(gL, "gL", 2)
    M = L.shape[0]
    if out is None:
        out = padded(M, M, L.device)
    nbytes = _lib.load().mgp_chol_backward_workspace_bytes(M)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, L.device)
    _lib.call("mgp_chol_backward", L.data_ptr(), _ld(L), LinvT.data_ptr(), _ld(LinvT), gL.data_ptr(), _ld(gL), M,
              out.data_ptr(), _ld(out), workspace.data_ptr(), workspace.numel(), _stream())
    return out


def kl_grad(q_mu, q_sqrt, num_data, g_q_mu, g_q_sqrt):
    """Fold -KL / num_data into the ELBO gradients (in place)."""
    M, K = q_mu.shape
    _lib.call("mgp_kl_grad", q_mu.data_ptr(), _ld(q_mu), q_sqrt.data_ptr(), _ld(q_sqrt), q_sqrt.stride(0), M, K,
              float(num_data), g_q_mu.data_ptr(), _ld(g_q_mu), g_q_sqrt.data_ptr(), _ld(g_q_sqrt),
              g_q_sqrt.stride(0), _stream())


def adam_step(theta, grad, m1, m2, t, lr, u=None, beta1=0.9, beta2=0.999, eps=1e-7, grad_sign=-1.0):
    """One TF-legacy Adam step on theta (2-D view [rows, cols] with leading dimension),
    gradient of the ELBO (grad_sign -1 minimises -ELBO); u: unconstrained softplus shadow."""
    rows, cols = theta.shape
    if grad.shape[-1] != cols:
        raise ValueError("gradient / parameter shape mismatch")
    _lib.call("mgp_adam_step", theta.data_ptr(), u.data_ptr() if u is not None else None, grad.data_ptr(),
              int(grad.dtype == torch.float64), _ld(grad), m1.data_ptr(), m2.data_ptr(), rows, cols, _ld(theta),
              float(lr), float(beta1), float(beta2), float(eps), int(t), float(grad_sign), _stream())


class AdamSet:
    """adam_step over a fixed list of parameter blocks in one launch (mgp_adam_step_set;
    bit-identical to one adam_step per block).  blocks: (theta 2-D view, m1, m2, u or
    None); the pointer arrays of the fixed state are built once."""

    def __init__(self, blocks):
        import ctypes
        n = len(blocks)
        if not 1 <= n <= 16:
            raise ValueError("AdamSet takes 1 .. 16 parameter blocks")
        P, I64 = ctypes.c_void_p * n, ctypes.c_int64 * n
        self.n = n
        self.shapes = [tuple(th.shape) for th, *_ in blocks]
        self.theta = P(*[th.data_ptr() for th, *_ in blocks])
        self.u = P(*[(u.data_ptr() if u is not None else None) for *_, u in blocks])
        self.m1 = P(*[m1.data_ptr() for _, m1, _, _ in blocks])
        self.m2 = P(*[m2.data_ptr() for _, _, m2, _ in blocks])
        self.rows = I64(*[s[0] for s in self.shapes])
        self.cols = I64(*[s[1] for s in self.shapes])
        self.ld = I64(*[_ld(th) for th, *_ in blocks])
        self._keep = blocks
        self._P, self._I64, self._I32 = P, I64, ctypes.c_int32 * n

    def step(self, grads, t, lr, beta1=0.9, beta2=0.999, eps=1e-7, grad_sign=-1.0):
        """grads: one 2-D gradient per block, in order (float32 or float64)."""
        if len(grads) != self.n:
            raise ValueError(f"AdamSet.step takes {self.n} gradients, got {len(grads)}")
        dev = self._keep[0][0].device
        for j, (gr, s) in enumerate(zip(grads, self.shapes)):
            # the kernel reads rows x cols at the gradient's leading dimension: every block must
            # match its parameter's shape exactly, be float32 / float64, row-contiguous and on
            # the parameters' device
            if tuple(gr.shape) != s:
                raise ValueError(f"gradient {j}: shape {tuple(gr.shape)} != parameter shape {s}")
            if gr.dtype not in (torch.float32, torch.float64):
                raise ValueError(f"gradient {j}: dtype {gr.dtype} (float32 or float64 expected)")
            if gr.numel() and (gr.stride(-1) != 1 or gr.device != dev):
                raise ValueError(f"gradient {j}: must be row-contiguous on {dev}")
        _lib.call("mgp_adam_step_set", self.n, self.theta, self.u, self._P(*[gr.data_ptr() for gr in grads]),
                  self._I32(*[int(gr.dtype == torch.float64) for gr in grads]), self._I64(*[_ld(gr) for gr in grads]),
                  self.m1, self.m2, self.rows, self.cols, self.ld, float(lr), float(beta1), float(beta2), float(eps),
                  int(t), float(grad_sign), _stream())


def gram(X, Y, N=None, alpha=1.0, tri=False, out=None, workspace=None):
    """out[i][j] = alpha * sum_n X[i][n] Y[j][n] (tri: lower triangle, zeros above)."""
    _check(X, "X", 2), _check(Y, "Y", 2)
    MI, MJ = X.shape[0], Y.shape[0]
    N = X.shape[1] if N is None else N
    dev = X.device
    if out is None:
        out = padded(MI, MJ, dev)
    nbytes = _lib.load().mgp_gram_workspace_bytes(MI, MJ, N, int(tri))
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    _lib.call("mgp_gram", X.data_ptr(), _ld(X), MI, Y.data_ptr(), _ld(Y), MJ, N, float(alpha), int(tri),
              out.data_ptr(), _ld(out), workspace.data_ptr(), workspace.numel(), _stream())
    return out


def split_rows_f16(X, bound, N=None, out=None):
    """X's row image for gram_x6(x_rows=...) (mgp_split_rows_f16): X [MI, >=N] f32, bound a float32
    device tensor >= max |X| (the scale mgp_gram_f16 would use)."""
    _check(X, "X", 2)
    M = X.shape[0]
    N = X.shape[1] if N is None else N
    nbytes = _lib.load().mgp_rows_f16_bytes(M, N)
    if out is None or out.numel() < nbytes:
        out = _ws(nbytes, X.device)
    _lib.call("mgp_split_rows_f16", X.data_ptr(), _ld(X), M, N, bound.data_ptr(), out.data_ptr(), out.numel(),
              _stream())
    return out


def gram_x6(X, Y, W=None, alpha=1.0, mode=0, N=None, out=None, workspace=None, bounds=None, x_rows=None):
    """out[b][i][j] = alpha * sum_n X[b][i][n] W[b][n] Y[b][j][n] at f32 accuracy on the bf16 MFMA.
    X [B, MI, >=N] / [MI, >=N] (Y likewise; a 2-D operand is shared by the batch); W [B, >=N] or None;
    mode 0 full, 1 lower triangle, 2 symmetric.  bounds = (x_bound, y_bound, w_bound) float32
    device tensors of max |X|, |Y|, |W| (w_bound None without W): the split-f16 variant
    (mgp_gram_f16).  x_rows: split_rows_f16(X, x_bound) of a 2-D X (with bounds, W and a 2-D Y):
    the same products with X's split done once (mgp_gram_f16_rows)."""
    X3 = X if X.dim() == 3 else X.unsqueeze(0)
    Y3 = Y if Y.dim() == 3 else Y.unsqueeze(0)
    B = max(X3.shape[0], Y3.shape[0], W.shape[0] if W is not None and W.dim() == 2 else 1)
    MI, MJ = X3.shape[1], Y3.shape[1]
    N = X3.shape[2] if N is None else N
    dev = X.device
    if out is None:
        out = padded(MI, MJ, dev, batch=B)
    sx = X3.stride(0) if X3.shape[0] > 1 else 0
    sy = Y3.stride(0) if Y3.shape[0] > 1 else 0
    sw = (W.stride(0) if W.dim() == 2 and W.shape[0] > 1 else 0) if W is not None else 0
    nbytes = _lib.load().mgp_gram_x6_workspace_bytes(MI, MJ, N, B, int(mode))
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    so = out.stride(0) if out.dim() == 3 else MI * _ld(out)
    if x_rows is not None:
        xb, yb, wb = bounds
        _lib.call("mgp_gram_f16_rows", x_rows.data_ptr(), x_rows.numel(), MI, Y3.data_ptr(), Y3.stride(1), MJ,
                  W.data_ptr(), sw, N, B, float(alpha), int(mode), out.data_ptr(), out.stride(-2), so,
                  xb.data_ptr(), yb.data_ptr(), wb.data_ptr(), workspace.data_ptr(), workspace.numel(), _stream())
        return out
    if bounds is not None:
        xb, yb, wb = bounds
        _lib.call("mgp_gram_f16", X3.data_ptr(), X3.stride(1), sx, MI, Y3.data_ptr(), Y3.stride(1), sy, MJ,
                  W.data_ptr() if W is not None else None, sw, N, B, float(alpha), int(mode), out.data_ptr(),
                  out.stride(-2), so, xb.data_ptr(), yb.data_ptr(), wb.data_ptr() if wb is not None else None,
                  workspace.data_ptr(), workspace.numel(), _stream())
        return out
    _lib.call("mgp_gram_x6", X3.data_ptr(), X3.stride(1), sx, MI, Y3.data_ptr(), Y3.stride(1), sy, MJ,
              W.data_ptr() if W is not None else None, sw, N, B, float(alpha), int(mode), out.data_ptr(),
              out.stride(-2), so, workspace.data_ptr(), workspace.numel(), _stream())
    return out


def conditional_backward_workspace_bytes(M, N, K):
    return int(_lib.load().mgp_conditional_backward_workspace_bytes(M, N, K))


def conditional_backward_prep(q_sqrt, l_bound, out=None):
    """The q_sqrt-only part of the C-images backward (L_k's image at scale l_bound, the
    transposed triangles) as a uint8 device buffer for conditional_backward_x6(...,
    prep=...) (mgp_conditional_backward_prep_f16c)."""
    _check(q_sqrt, "q_sqrt", 3)
    K, M, _ = q_sqrt.shape
    nbytes = _lib.load().mgp_conditional_backward_prep_bytes(M, K)
    if out is None or out.numel() < nbytes:
        out = _ws(nbytes, q_sqrt.device)
    _lib.call("mgp_conditional_backward_prep_f16c", q_sqrt.data_ptr(), _ld(q_sqrt), q_sqrt.stride(0), M, K,
              l_bound.data_ptr(), out.data_ptr(), out.numel(), _stream())
    return out


def conditional_backward_x6(Afr, A, q_sqrt, q_mu, LinvT, Gmu, Gv, M, N, out=None, workspace=None, fmt="x6",
                            cross=None, c_images=None, prep=None, t_bound=None):
    """Backward of one layer's conditional (see include/mgp_hip.h): returns dict of
    g_q_mu [M, K], g_q_sqrt [K, M, M], g_Kuf [M, N], g_Lm [M, M], g_var (float64 [1]).
    fmt: format of A's image Afr ("f16": mgp_conditional_backward_f16; with cross "f8",
    default config.expert_cross(), mgp_conditional_backward_f16x8 -- Afr then comes
    from trsm_stats_x6(..., A=..., cross="f8")).  c_images = (Cfr, colmax, l_bound) from
    expert_conditional_x6(..., c_out=...) (f16, cross "f16"): mgp_conditional_backward_f16c."""
    K = q_mu.shape[1]
    dev = q_mu.device
    if out is None:
        out = {"g_q_mu": padded(M, K, dev), "g_q_sqrt": padded(M, M, dev, batch=K),
               "g_Kuf": padded(M, N, dev), "g_Lm": padded(M, M, dev),
               "g_var": torch.empty(1, dtype=torch.float64, device=dev)}
    nbytes = _lib.load().mgp_conditional_backward_workspace_bytes(M, N, K)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    if _ld(Gmu) != _ld(Gv):
        raise ValueError("Gmu and Gv must share a leading dimension")
    o = out
    from .config import expert_cross
    entry = "mgp_conditional_backward_" + _fmt(fmt)
    if entry.endswith("f16") and (cross or expert_cross()) == "f8":
        entry += "x8"
    args = [Afr.data_ptr(), Afr.numel(), A.data_ptr(), _ld(A),
            q_sqrt.data_ptr(), _ld(q_sqrt), q_sqrt.stride(0), q_mu.data_ptr(), _ld(q_mu),
            LinvT.data_ptr(), _ld(LinvT), Gmu.data_ptr(), Gv.data_ptr(), _ld(Gmu), M, N, K,
            o["g_q_mu"].data_ptr(), _ld(o["g_q_mu"]), o["g_q_sqrt"].data_ptr(), _ld(o["g_q_sqrt"]),
            o["g_q_sqrt"].stride(0), o["g_Kuf"].data_ptr(), _ld(o["g_Kuf"]), o["g_Lm"].data_ptr(),
            _ld(o["g_Lm"]), o["g_var"].data_ptr(), workspace.data_ptr(), workspace.numel()]
    if c_images is not None:
        if entry != "mgp_conditional_backward_f16":
            raise ValueError("c_images need the split-f16 format with f16 cross terms")
        Cfr, colmax, l_bound = c_images
        entry = "mgp_conditional_backward_f16c"
        args += [Cfr.data_ptr(), Cfr.numel(), colmax.data_ptr(), l_bound.data_ptr()]
        if prep is not None:   # from conditional_backward_prep(q_sqrt, l_bound) of the same q_sqrt
            entry += "_prepped"   # t_bound: max |LinvT| (e.g. image_bound of K3's bounded L^-T image)
            args += [prep.data_ptr(), prep.numel(), t_bound.data_ptr() if t_bound is not None else None]
    elif prep is not None:
        raise ValueError("prep needs c_images (the C-images backward)")
    _lib.call(entry, *args, _stream())
    return out


def c_images_bytes(M, N, K):
    """Bytes of the C_k = L_k^T A images of expert_conditional_x6(..., c_out=...)."""
    return _lib.load().mgp_c_images_bytes(M, N, K)


def colnorm_max(q_sqrt, out=None):
    """max over experts and columns of ||tril(q_sqrt[k])[:, j]||_2 (float32 device [1])."""
    _check(q_sqrt, "q_sqrt", 3)
    if out is None:
        out = torch.empty(1, dtype=torch.float32, device=q_sqrt.device)
    K, M = q_sqrt.shape[0], q_sqrt.shape[1]
    _lib.call("mgp_colnorm_max", q_sqrt.data_ptr(), _ld(q_sqrt), q_sqrt.stride(0), M, K, out.data_ptr(), _stream())
    return out


def image_bound(img, M, K=None, N=None):
    """The device bound in a split image's trailer (float32 view [1]): lower images
    (K given) or column images (N given)."""
    lib = _lib.load()
    size = lib.mgp_x6_lower_bytes(M, K) if K is not None else lib.mgp_x6_cols_bytes(M, N)
    return img.view(torch.uint8)[size - 256:size - 252].view(torch.float32)


# --------------------------------------------------------------------------- K7
def gauss_kl_white(q_mu, q_sqrt, out=None, workspace=None):
    """Whitened KL (models.py:79) as a float64 device tensor of shape [1]."""
    _check(q_mu, "q_mu", 2), _check(q_sqrt, "q_sqrt", 3)
    q_sqrt = as_padded(q_sqrt)  # float4 rows (no copy for the layers' padded storage)
    M, K = q_mu.shape
    dev = q_mu.device
    if out is None:
        out = torch.empty(1, dtype=torch.float64, device=dev)
    nbytes = _lib.load().mgp_kl_workspace_bytes(M, K)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    _lib.call("mgp_gauss_kl_white", q_mu.data_ptr(), _ld(q_mu), q_sqrt.data_ptr(), _ld(q_sqrt),
              q_sqrt.stride(0), M, K, out.data_ptr(), workspace.data_ptr(), workspace.numel(),
              _stream())
    return out


# --------------------------------------------------------------------------- K6
def elbo_terms(mu_f, var_f, mu_a, var_a, Y, lik_var, S, tau=1e-2, noise=None, seed=0, n_offset=0,
               out=None, workspace=None, assign_lik_var=None, multiclass_eps=None, jitter=None):
    """Sum over local points of logsumexp_s(sum_k W ve) - log S (float64 [1]).
    With assign_lik_var: the SMGPModified data term (models.py:112-123).
    multiclass_eps: the pred likelihood is MultiClass(K) / RobustMax(eps) (lik_var unused)."""
    jitter = default_jitter() if jitter is None else jitter
    for t, n in ((mu_f, "mu_f"), (var_f, "var_f"), (mu_a, "mu_a"), (var_a, "var_a")):
        _check(t, n, 2)
    ldf = _ld(mu_f)
    if not (_ld(var_f) == _ld(mu_a) == _ld(var_a) == ldf):
        raise ValueError("conditional outputs must share a leading dimension")
    K, N = mu_f.shape
    dev = mu_f.device
    Y = Y.reshape(-1)
    _check(Y, "Y")
    if multiclass_eps is None:
        _check(lik_var, "lik_var")
    if Y.numel() != N or not Y.is_contiguous():
        raise ValueError("Y must be contiguous with N elements")
    if out is None:
        out = torch.empty(1, dtype=torch.float64, device=dev)
    nbytes = _lib.load().mgp_elbo_workspace_bytes(N)
    if workspace is None or workspace.numel() < nbytes:
        workspace = _ws(nbytes, dev)
    zp = up = None
    if noise is not None:
        z, u = noise
        _check(z, "noise_z", 3), _check(u, "noise_u", 3)
        if tuple(z.shape) != (S, N, K) or tuple(u.shape) != (S, N, K):
            raise ValueError("explicit noise must be [S, N, K]")
        z, u = z.contiguous(), u.contiguous()
        zp, up = z.data_ptr(), u.data_ptr()
    if multiclass_eps is not None:
        if assign_lik_var is not None:
            _check(assign_lik_var, "assign_lik_var")
        _lib.call("mgp_elbo_terms_multiclass", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(),
                  var_a.data_ptr(), ldf, Y.data_ptr(), float(multiclass_eps),
                  assign_lik_var.data_ptr() if assign_lik_var is not None else None, N, K, S, float(tau),
                  float(jitter), zp, up,
                  int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), out.data_ptr(), workspace.data_ptr(),
                  workspace.numel(), _stream())
        return out
    if assign_lik_var is not None:
        _check(assign_lik_var, "assign_lik_var")
        _lib.call("mgp_elbo_terms_modified", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(),
                  var_a.data_ptr(), ldf, Y.data_ptr(), lik_var.data_ptr(), assign_lik_var.data_ptr(), N, K,
                  S, float(tau), float(jitter), zp, up, int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), out.data_ptr(),
                  workspace.data_ptr(), workspace.numel(), _stream())
        return out
    _lib.call("mgp_elbo_terms", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(), var_a.data_ptr(),
              ldf, Y.data_ptr(), lik_var.data_ptr(), N, K, S, float(tau), float(jitter), zp, up,
              int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), out.data_ptr(), workspace.data_ptr(),
              workspace.numel(), _stream())
    return out


def elbo_combine(data_sum, kl_f, kl_a, n_batch, num_data, out=None, out64=None):
    dev = data_sum.device
    if out is None:
        out = torch.empty((), dtype=F32, device=dev)
    if out64 is None:
        out64 = torch.empty((), dtype=torch.float64, device=dev)
    _lib.call("mgp_elbo_combine", data_sum.data_ptr(), kl_f.data_ptr(), kl_a.data_ptr(),
              float(n_batch), float(num_data), out.data_ptr(), out64.data_ptr(), _stream())
    return out, out64


def predict_epilogue(fmean, fvar, amean, lik_var, want_y=True, want_assign=False):
    """[N, K] outputs: y mean/var (likelihoods.py:31-32) and softmax assignment."""
    ref = fmean if fmean is not None else amean
    K, N = ref.shape
    dev = ref.device
    ym = torch.empty(N, K, dtype=F32, device=dev) if want_y else None
    yv = torch.empty(N, K, dtype=F32, device=dev) if want_y else None
    asg = torch.empty(N, K, dtype=F32, device=dev) if want_assign else None
    _lib.call("mgp_predict_epilogue", fmean.data_ptr() if fmean is not None else None,
              fvar.data_ptr() if fvar is not None else None,
              amean.data_ptr() if amean is not None else None, _ld(ref),
              lik_var.data_ptr() if lik_var is not None else None, N, K,
              ym.data_ptr() if ym is not None else None, yv.data_ptr() if yv is not None else None,
              asg.data_ptr() if asg is not None else None, _stream())
    return ym, yv, asg


def philox_noise(seed, n_offset, N, K, S, device, want_z=True, want_u=True):
    z = torch.empty(S, N, K, dtype=F32, device=device) if want_z else None
    u = torch.empty(S, N, K, dtype=F32, device=device) if want_u else None
    _lib.call("mgp_philox_noise", int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), N, K, S,
              z.data_ptr() if z is not None else None, u.data_ptr() if u is not None else None,
              _stream())
    return z, u


def philox_normal2(seed, n_offset, N, K, S, device):
    z = torch.empty(S, N, K, dtype=F32, device=device)
    _lib.call("mgp_philox_normal2", int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), N, K, S,
              z.data_ptr(), _stream())
    return z


def predict_samples(mu_f, var_f, mu_a, var_a, lik_var, S, tau=1e-2, noise=None, seed=0,
                    n_offset=0, multiclass_eps=None, jitter=None):
    """samples_y, samples_f [S, N] (models.py:91-103); multiclass_eps: MultiClass / RobustMax
    predictive mean / variance for samples_y (lik_var unused)."""
    jitter = default_jitter() if jitter is None else jitter
    K, N = mu_f.shape
    dev = mu_f.device
    sy = torch.empty(S, N, dtype=F32, device=dev)
    sf = torch.empty(S, N, dtype=F32, device=dev)
    ptrs = [None, None, None]
    if noise is not None:
        noise = [t.contiguous() for t in noise]
        for t in noise:
            _check(t, "noise", 3)
            if tuple(t.shape) != (S, N, K):
                raise ValueError("explicit noise must be [S, N, K]")
        ptrs = [t.data_ptr() for t in noise]
    if multiclass_eps is not None:
        _lib.call("mgp_predict_samples_multiclass", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(),
                  var_a.data_ptr(), _ld(mu_f), float(multiclass_eps), N, K, S, float(tau), float(jitter), *ptrs,
                  int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), sy.data_ptr(), sf.data_ptr(), _stream())
        return sy, sf
    _lib.call("mgp_predict_samples", mu_f.data_ptr(), var_f.data_ptr(), mu_a.data_ptr(),
              var_a.data_ptr(), _ld(mu_f), lik_var.data_ptr(), N, K, S, float(tau), float(jitter), *ptrs,
              int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), sy.data_ptr(), sf.data_ptr(), _stream())
    return sy, sf


def multiclass_predict(fmean, fvar, epsilon):
    """MultiClass._predict_mean_and_var (GPflow 2.7): (ps, ps - ps^2), each [N, K]."""
    _check(fmean, "fmean", 2), _check(fvar, "fvar", 2)
    K, N = fmean.shape
    if _ld(fvar) != _ld(fmean):
        raise ValueError("fmean and fvar must share a leading dimension")
    ym = torch.empty(N, K, dtype=F32, device=fmean.device)
    yv = torch.empty(N, K, dtype=F32, device=fmean.device)
    _lib.call("mgp_multiclass_predict", fmean.data_ptr(), fvar.data_ptr(), _ld(fmean), N, K, float(epsilon),
              ym.data_ptr(), yv.data_ptr(), _stream())
    return ym, yv


# --------------------------------------------------------------------------- method-level API
def _latents_check(mu, var, name):
    _check(mu, "mu_" + name, 2), _check(var, "var_" + name, 2)
    if _ld(var) != _ld(mu) or var.shape != mu.shape:
        raise ValueError(f"mu_{name} and var_{name} must share shape and leading dimension")


def assign_logits(mu_a, var_a, S, N, stride_s=0, noise_z=None, seed=0, n_offset=0, jitter=None):
    """SMGP.W_dist's logits (models.py:56-59, utils.py:26-27): [S, N, K] =
    mu_a + z sqrt(var_a + jitter); mu_a / var_a expert-major [K, >= (S-1) stride_s + N]."""
    jitter = default_jitter() if jitter is None else jitter
    _latents_check(mu_a, var_a, "a")
    K = mu_a.shape[0]
    out = torch.empty(S, N, K, dtype=F32, device=mu_a.device)
    zp = None
    if noise_z is not None:
        _check(noise_z, "noise_z", 3)
        if tuple(noise_z.shape) != (S, N, K):
            raise ValueError("explicit noise must be [S, N, K]")
        noise_z = noise_z.contiguous()
        zp = noise_z.data_ptr()
    _lib.call("mgp_assign_logits", mu_a.data_ptr(), var_a.data_ptr(), _ld(mu_a), int(stride_s), N, K, S,
              float(jitter), zp, int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), out.data_ptr(), _stream())
    return out


def relaxed_onehot_sample(logits, S, N, tau=1e-2, noise_u=None, seed=0, n_offset=0):
    """RelaxedOneHotCategorical(tau, logits).sample() on logits [S * N, K] (rows s * N + n)."""
    _check(logits, "logits")
    K = logits.shape[-1]
    if logits.numel() != S * N * K:
        raise ValueError("logits must hold S * N rows of K")
    logits = logits.contiguous()
    W = torch.empty(S * N, K, dtype=F32, device=logits.device)
    up = None
    if noise_u is not None:
        _check(noise_u, "noise_u")
        if noise_u.numel() != S * N * K:
            raise ValueError("explicit noise must be [S, N, K]")
        noise_u = noise_u.contiguous()
        up = noise_u.data_ptr()
    _lib.call("mgp_relaxed_onehot_sample", logits.data_ptr(), N, K, S, float(tau), up,
              int(seed) & 0xFFFFFFFFFFFFFFFF, int(n_offset), W.data_ptr(), _stream())
    return W


def e_log_p_y(mu_f, var_f, Y, lik_var, W, S, N, stride_s=0, mu_a=None, var_a=None, assign_lik_var=None,
              multiclass_eps=None):
    """SMGP.E_log_p_Y (models.py:63-67; SMGPModified :112-123 with assign_lik_var) -> [N]."""
    _latents_check(mu_f, var_f, "f")
    K = mu_f.shape[0]
    Y = Y.reshape(-1)
    _check(Y, "Y"), _check(W, "W")
    if Y.numel() != N or not Y.is_contiguous():
        raise ValueError("Y must be contiguous with N elements")
    if W.numel() != S * N * K:
        raise ValueError("W must be [S, N, K]")
    W = W.contiguous()
    if multiclass_eps is None:
        _check(lik_var, "lik_var")
    if assign_lik_var is not None:
        _check(assign_lik_var, "assign_lik_var")
        _latents_check(mu_a, var_a, "a")
        if _ld(mu_a) != _ld(mu_f):
            raise ValueError("the two layers' latents must share a leading dimension")
    out = torch.empty(N, dtype=F32, device=mu_f.device)
    ptr = lambda t: t.data_ptr() if t is not None else None
    _lib.call("mgp_e_log_p_y", mu_f.data_ptr(), var_f.data_ptr(), ptr(mu_a), ptr(var_a), _ld(mu_f), int(stride_s),
              Y.data_ptr(), None if multiclass_eps is not None else lik_var.data_ptr(), ptr(assign_lik_var),
              float(multiclass_eps or 0.0), W.data_ptr(), N, K, S, out.data_ptr(), _stream())
    return out
