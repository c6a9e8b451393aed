"""SGP / SMGP / SMGPModified / SVGPModified on the MI355X kernels.

Drop-in counterparts of MixtureGPs/models.py (same class names, constructor
arguments and method names).  The SMGP ELBO hot path
(SMGP._build_likelihood, models.py:69-79) runs as:

  both layers (pred, assign) at once, default split-f16 format:   reference call site
    K2+K3 mgp_kuu_potrf_trtri_kuf   Kuu + jitter I built in     models.py:135, 141 (cholesky)
                                    float64, L and L^-1; the
                                    step launches also write
    K1                              both layers' Kuf images     models.py:139
          mgp_split_upper_f16_bounded_batch   L^-T images
          mgp_qsqrt_images_kl_f16_batch       tril(q_sqrt) images + K7 KL   models.py:79, 141-143
    K4 mgp_trsm_stats_f16_batch     A image + stats             models.py:141-143 (triangular_solve, A^T q_mu)
    K5 mgp_expert_conditional_f16_batch  fmean, fvar [K, N]     models.py:141-143 (LTA, fvar)
    (config expert_format "x6": the same chain on exact split-bf16 images, six bf16
     products per f32 product -- mgp_rbf_kuf_x6, mgp_split_upper_x6 / _lower_x6,
     mgp_trsm_stats_x6, mgp_expert_conditional_x6 -- csrc/split3.hip;
     config.set_conditional_mode("f32"): mgp_rbf_kuf + mgp_trsm_stats +
     mgp_expert_conditional_f32 on the exact-f32 MFMA)
  K6 mgp_elbo_terms         sum_n lse_s(...)        models.py:55-67,73-76
  mgp_elbo_combine          ELBO scalar             models.py:76,79

The reference evaluates every conditional on S tiled copies of X
(SGP.integrate, models.py:35-36); the copies are identical, so the conditional
is computed once per data point and S only enters the Monte-Carlo term.
Outputs that the reference returns with a leading S axis (predict_f on tiled
inputs, predict_y) are returned as broadcast views of that single result.

Compute dtype is float32 on the device; the parity tolerances against the
float64 reference semantics are stated in tests/.
"""
import math

import numpy as np
import torch

from . import ops
from .broadcasting_lik import BroadcastingLikelihood
from .config import (conditional_mode, default_device, default_jitter, expert_cross, expert_planes,
                     forward_image_format, step_schedule)

# both layers' K4, and both layers' K5, in one launch each in the step (False: one launch
# per layer and kernel; A/B probes only)
_K4_BATCHED = True
# the training forward's colnorm_max (the C_k images' bound) on the side stream beside K3
# (False: on the main stream right before K5; A/B probes only)
_COLMAX_SIDE = True
# split-f16: both layers' tril(q_sqrt) images and KL terms by mgp_qsqrt_images_kl_f16_batch
# (False: mgp_split_lower_f16 + mgp_gauss_kl_white per layer; A/B probes only)
_QS_BATCH = True
# k1_in_k3 carries K1's image blocks on the step launches' idle CUs at one 512-thread
# workgroup per CU; past this image size (N * M) the blocks outlast the chain's steps
# (BASELINE c5, N * M = 2^29: K3 2.15 -> 5.78 ms) and K1 runs on the side stream instead
# (schedule overlap, bit-identical)
_K1_IN_K3_MAX_NM = 1 << 27
_TAIL_BATCH = True   # both layers' Cholesky / RBF backward in one batch each (elbo_and_grad)
_RBF_NO_FILL = True  # the batched RBF backward overwrites gZ / g_ls (False: zero fills + accumulate; A/B only)
# training: the q_sqrt-only launches of the C-images backward (L_k's image, L_k^T) on the
# side stream beside K3 (mgp_conditional_backward_prep_f16c; False: inside the backward)
_COND_PREP = True
_T_BOUND = True   # the C-images backward takes max |LinvT| from K3's bounded L^-T images (A/B: False)

# The training step keeps each layer's C_k = L_k^T A images for the backward
# (mgp_conditional_backward_f16c) while both layers' sets fit in this fraction of the
# device's HBM (config 5: 2 x 51.5 GB of 288 GB); beyond it the backward rebuilds
# S_k = L_k L_k^T.  C_IMAGES_MAX_BYTES (per layer), when set, overrides it.
C_IMAGES_HBM_FRACTION = 0.4
C_IMAGES_MAX_BYTES = None
from .kernels import SquaredExponential
from .likelihoods import MultiClass

TAU = 1e-2  # RelaxedOneHotCategorical temperature, models.py:60


def _splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return x ^ (x >> 31)


class _Stage:
    """Optional HIP-event bracket around a stage, recorded on torch's current
    stream (the stream every libmgp_hip call of the model is launched on)."""

    def __init__(self, timing, name):
        self.timing, self.name = timing, name

    def __enter__(self):
        if self.timing is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()
        return self

    def __exit__(self, *exc):
        if self.timing is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.timing.setdefault(self.name, []).append((self.e0, e1))
        return False


class HostArray(np.ndarray):
    """Host float64 array returned by the public predict_* methods: what the
    reference's EagerTensors give the demos (numpy consumes it directly,
    demos/demo_tf2.py:63-72,86-87,98-99, and `.numpy()` works as on a TF tensor)."""

    def numpy(self):
        return np.asarray(self)


def _host(t):
    """Device result -> HostArray (float64, the reference's default_float)."""
    return t.detach().to(torch.float64).cpu().numpy().view(HostArray)


def _to_dev(x, device, dtype=torch.float32):
    t = torch.as_tensor(np.asarray(x) if not isinstance(x, torch.Tensor) else x)
    return t.to(device=device, dtype=dtype)


class SVGPModified:
    """Whitened SVGP layer with K latent GPs sharing one kernel and one Z
    (GPflow SVGP(kernel, likelihood, Z, num_latent_gps=K, whiten=True) with the
    posterior plugin IndependentPosteriorSingleOutputModified, models.py:126-160).

    Variational state: q_mu [M, K] (init zeros) and q_sqrt [K, M, M] lower
    triangular (init identity), as GPflow's SVGP initialises them."""

    def __init__(self, kernel, likelihood, inducing_variable, num_latent_gps=1, whiten=True,
                 q_mu=None, q_sqrt=None, q_diag=False, mean_function=None, device=None):
        if not whiten:
            raise NotImplementedError("only the whitened SVGP (whiten=True) is on the hot path")
        if q_diag:
            raise NotImplementedError("q_diag=True is not used by the reference models")
        if mean_function is not None:
            raise NotImplementedError("the reference layers use the Zero mean function")
        if not isinstance(kernel, SquaredExponential):
            raise TypeError("kernel must be modulatedgps_amd.kernels.SquaredExponential")
        self.device = torch.device(device or kernel.device or default_device())
        self.kernel = kernel
        self.likelihood = likelihood
        self.whiten = True
        Z = _to_dev(inducing_variable, self.device)
        if Z.dim() == 1:
            Z = Z[:, None]
        self.Z = Z.contiguous()
        self._last_info = None
        M = self.Z.shape[0]
        self.num_latent_gps = int(num_latent_gps)
        K = self.num_latent_gps
        self.q_mu = torch.zeros(M, K, dtype=torch.float32, device=self.device)
        self.q_sqrt = ops.padded(M, M, self.device, batch=K, zero=True)
        self.q_sqrt.copy_(torch.eye(M, device=self.device).expand(K, M, M))
        if q_mu is not None or q_sqrt is not None:
            self.set_variational(q_mu if q_mu is not None else self.q_mu,
                                 q_sqrt if q_sqrt is not None else self.q_sqrt)

    # ------------------------------------------------------------------ state
    @property
    def inducing_variable(self):
        return self.Z

    @property
    def num_inducing(self):
        return self.Z.shape[0]

    def set_variational(self, q_mu, q_sqrt):
        """Set q_mu [M, K] and q_sqrt [K, M, M] (band_part(-1, 0) is applied)."""
        q_mu = _to_dev(q_mu, self.device)
        q_sqrt = _to_dev(q_sqrt, self.device)
        M, K = self.num_inducing, self.num_latent_gps
        if tuple(q_mu.shape) != (M, K) or tuple(q_sqrt.shape) != (K, M, M):
            raise ValueError(f"expected q_mu [{M},{K}] and q_sqrt [{K},{M},{M}]")
        self.q_mu.copy_(q_mu)
        self.q_sqrt.copy_(torch.tril(q_sqrt))

    def parameters(self):
        return {"Z": self.Z, "q_mu": self.q_mu, "q_sqrt": self.q_sqrt, **self.kernel.parameters()}

    # ------------------------------------------------------------------ ops
    def Kuu(self, out=None):
        return ops.rbf_kuu(self.Z, self.kernel.variance, self.kernel.lengthscales, default_jitter(),
                           out=out)

    def factorise(self, want_L=False):
        """Kuu (float64) -> L, (L^-1)^T (float32 [1, M, M]) and info (models.py:135,141)."""
        return ops.kuu_potrf_trtri([self.Z], [self.kernel.variance], [self.kernel.lengthscales],
                                   default_jitter(), want_L=want_L)

    def prior_kl(self, out=None):
        """GPflow SVGP.prior_kl -> gauss_kl(q_mu, q_sqrt) whitened (models.py:79); float64 [1]."""
        return ops.gauss_kl_white(self.q_mu, self.q_sqrt, out=out)

    def operand_images(self, X, bufs=None, timing=None, fmt="x6"):
        """x6 mode: the split-bf16 images that do not depend on the Cholesky --
        Kuf (K1) and tril(q_sqrt) (split-f16 when fmt == "f16") -- so a caller
        can build them on a side stream while K3 runs.  Returns (Kfr, Lfr)."""
        bufs = bufs or {}
        X = self.kernel._x(X)
        with _Stage(timing, "rbf_kuf"):
            Kfr = ops.rbf_kuf_x6(X, self.Z, self.kernel.variance, self.kernel.lengthscales,
                                 out=bufs.get("Kfr"), fmt=fmt)
        with _Stage(timing, "split_tri"):
            Lfr = ops.split_lower_x6(self.q_sqrt, out=bufs.get("Lfr"), fmt=fmt)
        return Kfr, Lfr

    def conditional_kn(self, X, LinvT=None, bufs=None, timing=None, images=None, fmt=None):
        """Whitened conditional for X [N, D]: fmean, fvar as expert-major [K, N] views.

        LinvT: (L^-1)^T of this layer's Kuu if already factorised (the SMGP
        factorises both layers in one batched sweep).  images: (Kfr, Lfr) from
        operand_images (x6 mode), if already built."""
        X = self.kernel._x(X)
        if LinvT is None:
            _, LinvT, info = self.factorise()
            self._last_info = info
            LinvT = LinvT[0]
        bufs = bufs or {}
        fmt = fmt or forward_image_format()
        if conditional_mode() == "x6":
            Kfr, Lfr = images if images is not None else self.operand_images(X, bufs, timing, fmt)
        else:
            with _Stage(timing, "rbf_kuf"):
                Kuf = ops.rbf_kuf(X, self.Z, self.kernel.variance, self.kernel.lengthscales,
                                  out=bufs.get("Kuf"))
        if conditional_mode() == "f32":
            with _Stage(timing, "trsm_stats"):
                A, stats = ops.trsm_stats(LinvT, Kuf, self.q_mu, A=bufs.get("A"),
                                          stats=bufs.get("stats"))
            with _Stage(timing, "expert_cond"):
                return ops.expert_conditional(A, self.q_sqrt, stats, self.kernel.variance,
                                              fmean=bufs.get("fmean"), fvar=bufs.get("fvar"),
                                              workspace=bufs.get("ws_expert"))
        Afr, stats = self.x6_trsm(X.shape[0], LinvT, Kfr, bufs, timing, fmt)
        return self.x6_expert(X.shape[0], Afr, Lfr, stats, bufs, timing, fmt)

    def x6_trsm(self, N, LinvT, Kfr, bufs, timing=None, fmt="x6", Tfr=None):
        """K4 on images: A's image (split-f16 when fmt == "f16") and the column
        statistics (x6 mode).  Tfr: L^-T's image if already split."""
        if Tfr is None:
            with _Stage(timing, "split_tri"):
                Tfr = ops.split_upper_x6(LinvT, out=bufs.get("Tfr"), fmt=fmt)
        with _Stage(timing, "trsm_stats"):
            return ops.trsm_stats_x6(Tfr, Kfr, self.q_mu, self.num_inducing, N, Afr=bufs.get("Afr"),
                                     stats=bufs.get("stats"), A=bufs.get("A32"),
                                     f16_variance=self.kernel.variance if fmt == "f16" else None, in_fmt=fmt)

    def x6_expert(self, N, Afr, Lfr, stats, bufs, timing=None, fmt="x6", colmax_ready=False):
        """K5 on images: fmean, fvar [K, N] (x6 mode).  colmax_ready: the C_k images'
        column bound (colnorm_max of q_sqrt) is already in bufs["c_out"][1]."""
        with _Stage(timing, "expert_cond"):
            c_out = bufs.get("c_out")  # training (split-f16): C_k images for the backward
            if c_out is not None and not colmax_ready:
                ops.colnorm_max(self.q_sqrt, out=c_out[1])
            return ops.expert_conditional_x6(Afr, Lfr, stats, self.kernel.variance, self.num_inducing, N,
                                             self.num_latent_gps, fmean=bufs.get("fmean"),
                                             fvar=bufs.get("fvar"), workspace=bufs.get("ws_expert"),
                                             planes=expert_planes(), fmt=fmt, c_out=c_out)

    def conditional_experts(self, X, k0, k1, LinvT=None):
        """fmean, fvar [k1 - k0, N] of experts k0 .. k1 - 1 only (the expert-parallel
        layout: each rank owns a range of the K experts).  Kuf, the
        Cholesky and A are shared by all experts and computed in full; K4's
        statistics and K5 run on the expert range (q_mu columns, q_sqrt batch)."""
        X = self.kernel._x(X)
        M, N = self.num_inducing, X.shape[0]
        if not (0 <= k0 <= k1 <= self.num_latent_gps):
            raise ValueError("invalid expert range")
        if LinvT is None:
            _, LinvT, info = self.factorise()
            self._last_info = info
            LinvT = LinvT[0]
        fmt = forward_image_format()
        Kfr = ops.rbf_kuf_x6(X, self.Z, self.kernel.variance, self.kernel.lengthscales, fmt=fmt)
        Tfr = ops.split_upper_x6(LinvT, fmt=fmt)
        Afr, stats = ops.trsm_stats_x6(Tfr, Kfr, self.q_mu[:, k0:k1], M, N,
                                       f16_variance=self.kernel.variance if fmt == "f16" else None, in_fmt=fmt)
        Lfr = ops.split_lower_x6(self.q_sqrt[k0:k1], fmt=fmt)
        return ops.expert_conditional_x6(Afr, Lfr, stats, self.kernel.variance, M, N, k1 - k0,
                                         planes=expert_planes(), fmt=fmt)

    def _marginals_kn(self, Xnew, tiled=None):
        """Xnew [..., N, D] -> (fmean, fvar, S, N, stride_s, lead): expert-major [K, cols]
        marginals where sample s of point n is column s * stride_s + n.  S tiled copies
        of one input (SGP.integrate, models.py:35-36) are computed once (stride_s = 0).
        tiled=None recognises tiling without a device sync: a device tensor whose sample
        axis has stride 0 (what integrate() returns, an expand() view), or a host array
        whose copies compare equal on the host; a materialised device copy of tiled
        rows (X[None].repeat(S, 1, 1), tf.tile's result) is then computed row by row (the
        same values, S times the work and buffers).  tiled=True: the caller asserts the
        S copies are equal and copy 0 is computed once (no check, no sync); tiled=False:
        every row is computed."""
        host_tiled = False
        if tiled is not None:
            if not isinstance(Xnew, torch.Tensor):
                Xnew = torch.as_tensor(np.asarray(Xnew))
            host_tiled = bool(tiled) and Xnew.dim() >= 3
        elif not isinstance(Xnew, torch.Tensor):
            Xh = np.asarray(Xnew)
            if Xh.ndim >= 3:
                Xh2 = Xh.reshape(-1, *Xh.shape[-2:])
                host_tiled = Xh2.shape[0] > 1 and bool((Xh2 == Xh2[:1]).all())
        elif Xnew.dim() >= 3:
            lead_t = Xnew.shape[:-2]
            if Xnew.device.type == "cpu":
                X2 = Xnew.reshape(-1, *Xnew.shape[-2:])
                host_tiled = X2.shape[0] > 1 and bool(torch.equal(X2, X2[:1].expand_as(X2)))
            else:
                host_tiled = all(st == 0 for st, n in zip(Xnew.stride()[:len(lead_t)], lead_t) if n > 1)
        X = self.kernel._x(Xnew) if not host_tiled else None
        if host_tiled:
            Xsrc = Xnew if isinstance(Xnew, torch.Tensor) else torch.as_tensor(np.asarray(Xnew))
            lead, N = Xsrc.shape[:-2], Xsrc.shape[-2]
            S = int(np.prod(lead)) if len(lead) else 1
            fm, fv = self.conditional_kn(Xsrc[(0,) * len(lead)])
            return fm, fv, S, N, 0, lead
        if X.dim() == 2:
            fm, fv = self.conditional_kn(X)
            return fm, fv, 1, X.shape[0], 0, ()
        lead, N = X.shape[:-2], X.shape[-2]
        S = X.reshape(-1, N, X.shape[-1]).shape[0]
        fm, fv = self.conditional_kn(X.reshape(-1, X.shape[-1]))
        return fm, fv, S, N, N, lead

    def posterior(self, precompute_cache=None):
        """SVGPModified.posterior (models.py:148-160): the posterior plugin object whose
        _conditional_fused runs K1-K5 on this layer's current state (a NOCACHE-style
        view: the variational parameters are read at call time, whatever the cache type)."""
        return IndependentPosteriorSingleOutputModified(
            self.kernel, self.inducing_variable, self.q_mu, self.q_sqrt, whiten=self.whiten,
            mean_function=None, precompute_cache=precompute_cache, layer=self)

    @property
    def trainable_variables(self):
        """GPflow Module.trainable_variables of the layer: Z, q_mu, q_sqrt, kernel variance
        and lengthscales (device tensors holding the constrained values)."""
        return (self.Z, self.q_mu, self.q_sqrt, self.kernel.variance, self.kernel.lengthscales)

    def predict_f(self, Xnew, full_cov=False, full_output_cov=False, tiled=None):
        """GPflow SVGP.predict_f(Xnew): posterior(NOCACHE).fused_predict_f, i.e. the
        Modified posterior's _conditional_fused (models.py:129-144).
        Xnew [..., N, D] -> mean, var [..., N, K].  tiled: see _marginals_kn."""
        return self.posterior(PrecomputeCacheType.NOCACHE).fused_predict_f(Xnew, full_cov, full_output_cov,
                                                                          tiled=tiled)


class PrecomputeCacheType:
    """gpflow.posteriors.PrecomputeCacheType (TENSOR / VARIABLE / NOCACHE)."""
    TENSOR = "tensor"
    VARIABLE = "variable"
    NOCACHE = "nocache"


class IndependentPosteriorSingleOutputModified:
    """The reference's posterior plugin (models.py:126-144): GPflow's IndependentPosterior
    with _conditional_fused overridden to Knn = K_diag, Kmm = Kuu + jitter,
    Kmn = K(Z, Xnew), base_conditional(white=True).  Here _conditional_fused is the
    K1 -> K3 -> K4 -> K5 chain of the layer it was made from (SVGPModified.posterior)."""

    def __init__(self, kernel, inducing_variable, q_mu, q_sqrt, whiten=True, mean_function=None,
                 precompute_cache=None, layer=None):
        if not whiten:
            raise NotImplementedError("only the whitened posterior is on the hot path")
        if mean_function is not None:
            raise NotImplementedError("the reference layers use the Zero mean function")
        if layer is None:
            raise ValueError("the posterior runs on an SVGPModified layer's kernels (layer=...)")
        self.kernel, self.X_data, self.q_mu, self.q_sqrt = kernel, inducing_variable, q_mu, q_sqrt
        self.whiten, self.mean_function = whiten, mean_function
        self.cache_type = precompute_cache
        self._layer = layer

    def _conditional_fused(self, Xnew, full_cov=False, full_output_cov=False, tiled=None):
        """(fmean, fvar) [..., N, K] of the whitened SVGP marginals (models.py:129-144).
        tiled (extension): True when the caller's [S, N, D] input holds S equal copies
        (computed once without a check), False to compute every row, None to detect
        (SVGPModified._marginals_kn)."""
        if full_cov or full_output_cov:
            raise NotImplementedError("full_cov predictions are not used by the SMGP path")
        fm, fv, S, N, stride, lead = self._layer._marginals_kn(Xnew, tiled=tiled)
        K = fm.shape[0]
        shape = (*lead, N, K)
        if stride == 0 and len(lead):
            return fm.t().expand(shape), fv.t().expand(shape)
        return fm.t().reshape(shape), fv.t().reshape(shape)

    def fused_predict_f(self, Xnew, full_cov=False, full_output_cov=False, tiled=None):
        """GPflow BasePosterior.fused_predict_f: _conditional_fused + the (Zero) mean function."""
        return self._conditional_fused(Xnew, full_cov, full_output_cov, tiled=tiled)

    def predict_f(self, Xnew, full_cov=False, full_output_cov=False, tiled=None):
        return self.fused_predict_f(Xnew, full_cov, full_output_cov, tiled=tiled)


class RelaxedOneHotCategorical:
    """tfp.distributions.RelaxedOneHotCategorical(temperature, logits) as SMGP.W_dist
    returns it (models.py:60): logits [S * N, K] on the device; sample() runs the
    Gumbel-softmax kernel.  The first sample uses the key the logits were drawn with,
    so W_dist(Xt) -> sample(1) -> E_log_p_Y reproduces _build_likelihood with that key."""

    def __init__(self, temperature, logits, rows, seed=None, n_offset=0, model=None):
        self.temperature = float(temperature)
        self.logits = logits
        self._S, self._N = rows
        self._seed = seed
        self._model = model
        self._n_offset = int(n_offset)
        self._draws = 0

    def sample(self, sample_shape=(), noise_u=None, seed=None):
        """TFP sample semantics: sample() -> [S * N, K], sample(n) / sample((n,)) ->
        [n, S * N, K] relaxed one-hot samples (the reference draws sample(1)[0],
        models.py:73).  noise_u: explicit uniforms [n?, S, N, K].  Without noise and
        seed, the first draw uses the key the logits were drawn with (W_dist's, so
        W_dist -> sample(1) -> E_log_p_Y reproduces _build_likelihood with that key)
        and every later draw a fresh key from the model (TF's stateful RNG advances
        per call); with W_dist(noise_z=...) and no seed every draw is fresh."""
        shape = tuple(sample_shape) if isinstance(sample_shape, (tuple, list)) else (int(sample_shape),)
        n = int(np.prod(shape)) if shape else 1
        if n == 0:   # TFP: an empty sample, no draw (the RNG stream does not advance)
            return self.logits.new_empty((*shape, *self.logits.shape))
        outs = []
        for i in range(n):
            u = None
            if noise_u is not None:
                u = noise_u[i] if noise_u.dim() == 4 else noise_u
            if seed is not None:
                key = _splitmix64(int(seed) + i) if i else int(seed)
            elif self._draws == 0 and self._seed is not None:
                key = self._seed
            elif self._model is not None:
                key = self._model.next_seed()
            else:
                key = _splitmix64((self._seed or 0) * 0x100000001B3 + 0x5EED + self._draws)
            self._draws += 1
            outs.append(ops.relaxed_onehot_sample(self.logits, self._S, self._N, self.temperature, noise_u=u,
                                                  seed=key, n_offset=self._n_offset))
        if not shape:
            return outs[0]
        return torch.stack(outs).reshape(*shape, *outs[0].shape)


class SGP:
    """Scalable GP: X -> Xt = integrate(X) -> GP -> Y (models.py:23-41)."""

    def __init__(self, likelihood, pred_layer, num_samples=1, num_data=None):
        self.num_samples = int(num_samples)
        self.num_data = num_data
        self.likelihood = BroadcastingLikelihood(likelihood)
        self.pred_layer = pred_layer

    def integrate(self, X, S=1):
        """models.py:35-36 (kept for API parity; the hot path never tiles)."""
        X = torch.as_tensor(X)
        return X[None].expand(S, *X.shape), None

    def _mc_eps(self):
        """RobustMax epsilon when the pred likelihood is MultiClass, else None."""
        lik = self.likelihood.likelihood
        return lik.invlink.epsilon if isinstance(lik, MultiClass) else None

    def predict_y(self, Xnew, S=1):
        """models.py:38-41 -> (mean, var) [S, N, K] host arrays (HostArray, float64; S
        copies); the likelihood's _predict_mean_and_var through BroadcastingLikelihood
        (broadcasting_lik.py:44-46): Gaussian (mu, var + sigma^2) or MultiClass (ps, ps - ps^2).
        predict_y_device returns the same as float32 device views."""
        ym, yv = self.predict_y_device(Xnew, S)
        self.check_linalg(self.pred_layer._last_info)
        return _host(ym), _host(yv)

    def check_linalg(self, info=None):
        """Raise MGPLinAlgError if the last Cholesky of Kuu (both layers' for an SMGP
        evaluation) found a non-positive pivot -- the reference's InvalidArgumentError
        from base_conditional (models.py:141).  Reads K3's device `info` back (one host
        sync): run_adam does it at its ELBO readback, predict_* before returning."""
        info = getattr(self, "last_info", None) if info is None else info
        if info is not None:
            ops.check_info(info)

    def predict_y_device(self, Xnew, S=1):
        """predict_y as float32 device tensors [S, N, K] (broadcast views, no host copy)."""
        lik = self.likelihood.likelihood
        X = self.pred_layer.kernel._x(Xnew)
        fm, fv = self.pred_layer.conditional_kn(X)
        if self._mc_eps() is not None:
            ym, yv = ops.multiclass_predict(fm, fv, self._mc_eps())
        else:
            ym, yv, _ = ops.predict_epilogue(fm, fv, None, lik.variance.reshape(-1), want_y=True)
        return ym[None].expand(S, *ym.shape), yv[None].expand(S, *yv.shape)


class SMGP(SGP):
    """Mixture of Gaussian processes (models.py:44-103)."""

    def __init__(self, likelihood, pred_layer, assign_layer, K=3, num_samples=1, num_data=None,
                 seed=0):
        SGP.__init__(self, likelihood, pred_layer, num_samples, num_data)
        self.assign_layer = assign_layer
        self.K = int(K)
        if pred_layer.num_latent_gps != self.K or assign_layer.num_latent_gps != self.K:
            raise ValueError("both layers must have num_latent_gps == K")
        if isinstance(likelihood, MultiClass) and likelihood.num_classes != self.K:
            raise ValueError("a MultiClass pred likelihood needs num_classes == K (one latent GP per class)")
        self.device = pred_layer.device
        self.seed = int(seed)
        self._draws = 0
        self._bufs = {}
        self.last_info = None

    # ------------------------------------------------------------------ internals
    def _buffers(self, N, train=False):
        # the image formats decide which buffers exist (e.g. the C_k images of the
        # split-f16 training step), so a format switch between calls gets its own set
        key = (N, conditional_mode(), bool(train), forward_image_format(train), expert_cross())
        b = self._bufs.get(key)
        if b is not None:
            return b
        dev = self.device
        Mf, Ma, K = self.pred_layer.num_inducing, self.assign_layer.num_inducing, self.K
        Mx = max(Mf, Ma)
        T = ops.stats_tiles(Mx)
        x6 = conditional_mode() == "x6"
        kuf = None if x6 else ops.padded(Mx, N, dev)
        a = None if x6 else ops.padded(Mx, N, dev)
        st = ops.padded(2 * T * (K + 1), N, dev)  # per layer (the layers' K4 may run concurrently)
        cond = ops.padded(4 * K, N, dev)          # mu_f, var_f, mu_a, var_a
        b = {
            "Kuf_f": None if x6 else kuf[:Mf], "Kuf_a": None if x6 else kuf[:Ma],
            "A_f": None if x6 else a[:Mf], "A_a": None if x6 else a[:Ma],
            "stats_f": st[:ops.stats_tiles(Mf) * (K + 1)].unflatten(0, (-1, K + 1)),
            "stats_a": st[T * (K + 1):(T + ops.stats_tiles(Ma)) * (K + 1)].unflatten(0, (-1, K + 1)),
            "mu_f": cond[0:K], "var_f": cond[K:2 * K], "mu_a": cond[2 * K:3 * K],
            "var_a": cond[3 * K:4 * K],
            "kl": torch.empty(2, dtype=torch.float64, device=dev),
            "data_sum": torch.empty(1, dtype=torch.float64, device=dev),
            "elbo": torch.empty((), dtype=torch.float32, device=dev),
            "elbo64": torch.empty((), dtype=torch.float64, device=dev),
            "ws_expert": torch.empty(max(ops.expert_workspace_bytes(Mx, N, K),
                                         ops.expert_x6_workspace_bytes(Mx, N, K)), dtype=torch.uint8,
                                     device=dev),
        }
        if x6 and Mf == Ma and forward_image_format(train) == "f16" and expert_cross() == "f16":
            # the second layer's K5 workspace, only where both layers' K5 can run as one
            # launch (split-f16 images with f16 cross terms, equal M)
            b["ws_expert2"] = torch.empty_like(b["ws_expert"])
        if x6:  # split-bf16 images: Kuf / tril(q_sqrt) per layer (built on the side
            # stream while K3 runs), A and L^-T shared by the layers (processed in turn)
            for L in ("f", "a"):
                b["Kfr_" + L] = torch.empty(ops.x6_cols_bytes(Mx, N), dtype=torch.uint8, device=dev)
                b["Lfr_" + L] = torch.empty(ops.x6_lower_bytes(Mx, K), dtype=torch.uint8, device=dev)
            for L in ("f", "a"):  # per layer: the two layers' K4 run concurrently
                b["Afr_" + L] = torch.empty(ops.x6_cols_bytes(Mx, N), dtype=torch.uint8, device=dev)
                b["Tfr_" + L] = torch.empty(ops.x6_lower_bytes(Mx, 1), dtype=torch.uint8, device=dev)
        b["x6"] = x6
        if Mf == Ma and self.pred_layer.Z.shape[1] == self.assign_layer.Z.shape[1]:
            b["LinvT2"] = ops.padded(Mf, Mf, dev, batch=2)
        b["train"] = bool(train)
        if train:
            if not x6:
                raise NotImplementedError("the training step runs on the x6 conditional path")
            if "LinvT2" in b:
                b["L2"] = ops.padded(Mf, Mf, dev, batch=2)
            for L, M in (("f", Mf), ("a", Ma)):  # kept for the backward pass
                b["A32_" + L] = ops.padded(M, N, dev)
            b["G"] = ops.padded(4 * K, N, dev).unflatten(0, (4, K))
            cb = ops.c_images_bytes(Mx, N, K)
            limit = (C_IMAGES_MAX_BYTES if C_IMAGES_MAX_BYTES is not None else
                     C_IMAGES_HBM_FRACTION * torch.cuda.get_device_properties(dev).total_memory / 2)
            if forward_image_format(True) == "f16" and expert_cross() == "f16" and cb <= limit:
                for L in ("f", "a"):  # K5 writes C_k per expert; the backward reads them
                    b["Cfr_" + L] = torch.empty(cb, dtype=torch.uint8, device=dev)
                    b["colmax_" + L] = torch.empty(1, dtype=torch.float32, device=dev)
                    b["cprep_" + L] = torch.empty(ops._lib.load().mgp_conditional_backward_prep_bytes(Mx, K),
                                                  dtype=torch.uint8, device=dev)
            b["ws_cbwd"] = torch.empty(ops.conditional_backward_workspace_bytes(Mx, N, K), dtype=torch.uint8,
                                       device=dev)
        self._bufs[key] = b
        return b

    def _factorise(self, b, prep_event=None, tfr_bounds=False, kuf=None):
        """Kuu of both layers and their batched Cholesky + inverse (one K3 sweep).
        Training buffers also keep L (b["L_f"], b["L_a"]) for the backward pass.
        prep_event: recorded once Kuu is built (batched path only; else after K3).
        tfr_bounds: K3 also writes max |LinvT| into the L^-T split-f16 images'
        trailers (b["Tfr_f"], b["Tfr_a"]; batched path), for bounded splits.
        kuf: (X, fmt) -- K3's step launches also write both layers' Kuf images
        (b["Kfr_f"], b["Kfr_a"]; batched path, schedule "k1_in_k3")."""
        pf, pa = self.pred_layer, self.assign_layer
        train = b.get("train", False)
        if "LinvT2" in b:
            if pf.Z.stride(0) != pa.Z.stride(0):
                pa.Z = pa.Z.contiguous()
                pf.Z = pf.Z.contiguous()
            Lo, LinvT, info = ops.kuu_potrf_trtri(
                [pf.Z, pa.Z], [pf.kernel.variance, pa.kernel.variance],
                [pf.kernel.lengthscales, pa.kernel.lengthscales], default_jitter(), LinvT=b["LinvT2"],
                L=b.get("L2"), want_L=train, prep_event=prep_event,
                tfr_bound_images=[b["Tfr_f"], b["Tfr_a"]] if tfr_bounds else None,
                kuf=(kuf[0], [b["Kfr_f"], b["Kfr_a"]], kuf[1]) if kuf is not None else None)
            self.last_info = info
            if train:
                b["L_f"], b["L_a"] = Lo[0], Lo[1]
            b["LinvT_f"], b["LinvT_a"] = LinvT[0], LinvT[1]
            return LinvT[0], LinvT[1]
        outs = []
        infos = []
        for name, layer in (("f", pf), ("a", pa)):
            Lo, LinvT, info = layer.factorise(want_L=train)
            outs.append(LinvT[0])
            infos.append(info)
            if train:
                b["L_" + name] = Lo[0]
            b["LinvT_" + name] = LinvT[0]
        self.last_info = torch.cat(infos)
        if prep_event is not None:
            prep_event.record()
        return outs[0], outs[1]

    def _prep_event(self):
        """The K3 prep-done event (created once: its handle is passed to the C-ABI)."""
        if getattr(self, "_prep_ev", None) is None:
            self._prep_ev = torch.cuda.Event()
            self._prep_ev.record()   # creates the underlying hipEvent_t
        return self._prep_ev

    def _side_stream(self):
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def conditionals(self, X, timing=None, kl_out=None, train=False):
        """(mu_f, var_f, mu_a, var_a), each an expert-major [K, N] device view.

        x6 mode: K1 and the tril(q_sqrt) images of both layers (and, when kl_out
        is given, both KL terms) run on a side stream concurrently with the
        latency-bound K3 sweep, which occupies only a few CUs.  They start once
        K3 has built Kuu (its prep event): launched beside the build, K1's 4096
        workgroups starve it (101 us instead of ~20)."""
        X = self.pred_layer.kernel._x(X)
        N = X.shape[0]
        b = self._buffers(N, train)
        layers = (("f", self.pred_layer), ("a", self.assign_layer))
        images = {}
        fmt = forward_image_format(train)
        prep = None
        if b["x6"]:
            main = torch.cuda.current_stream(self.device)
            side = self._side_stream()
            prep = self._prep_event()
        # split-f16 L^-T images: K3 folds their scale bound (max |LinvT|) into its
        # writes of the inverse, so the split needs no reduction launches
        bounded = b["x6"] and "Tfr_a" in b and "LinvT2" in b and fmt == "f16"
        b["lt_bounded"] = bounded   # the backward takes max |LinvT| from the Tfr trailers
        sched = step_schedule() if (b["x6"] and "Tfr_a" in b) else "overlap"
        # schedule k1_in_k3: both layers' K1 as a side job of K3's step launches (batched K3)
        k1_in_k3 = (sched == "k1_in_k3" and "LinvT2" in b and self.pred_layer.kernel._x(X) is X
                    and self.assign_layer.kernel._x(X) is X
                    and N * self.pred_layer.num_inducing <= _K1_IN_K3_MAX_NM)
        if sched == "k1_in_k3" and not k1_in_k3:
            sched = "overlap"
        with _Stage(timing, "kuu_chol"):
            LinvT_f, LinvT_a = self._factorise(b, prep_event=prep, tfr_bounds=bounded,
                                               kuf=(X, fmt) if k1_in_k3 else None)
        Tfr = {}
        if b["x6"] and "Tfr_a" in b:
            # L^-T images straight after K3 on its stream (no cross-stream wait in front)
            with _Stage(timing, "split_tri"):
                if bounded and _K4_BATCHED:   # both layers' L^-T images in one launch (bit-identical)
                    Tfr["f"], Tfr["a"] = ops.split_upper_f16_bounded_batch(b["LinvT2"], [b["Tfr_f"], b["Tfr_a"]])
                else:
                    for L, lt in (("f", LinvT_f), ("a", LinvT_a)):
                        Tfr[L] = ops.split_upper_x6(lt, out=b["Tfr_" + L], fmt=fmt, bounded=bounded)
        late = {"k1_in_k3": (), "overlap": (), "k1a_late": ("a",), "k1a_k5": ("a",), "k1_main": ("f", "a"),
                "serial": ("f", "a")}[sched]
        if b["x6"]:
            pf, pa = self.pred_layer, self.assign_layer
            # split-f16: both layers' tril(q_sqrt) images and KL terms in three launches
            # (mgp_qsqrt_images_kl_f16_batch) instead of five per layer, beside K3's chain
            # (the batch entry also needs equal q_mu leading dimensions and q_sqrt ld / stride(0),
            # else the per-layer launches run)
            q_batch = (_QS_BATCH and fmt == "f16" and pf.q_mu.shape == pa.q_mu.shape and "Lfr_f" in b
                       and pf.q_mu.stride() == pa.q_mu.stride()
                       and pf.q_sqrt.stride() == pa.q_sqrt.stride())

            def side_work():
                for L, layer in layers:
                    X_ = layer.kernel._x(X)
                    if L not in late and not k1_in_k3:
                        with _Stage(timing, "rbf_kuf"):
                            ops.rbf_kuf_x6(X_, layer.Z, layer.kernel.variance, layer.kernel.lengthscales,
                                           out=b["Kfr_" + L], fmt=fmt)
                    with _Stage(timing, "split_tri"):
                        if not q_batch:
                            ops.split_lower_x6(layer.q_sqrt, out=b["Lfr_" + L], fmt=fmt)
                        if _COLMAX_SIDE and "colmax_" + L in b:   # training: the C_k bound, off the K3 -> K5 path
                            ops.colnorm_max(layer.q_sqrt, out=b["colmax_" + L])
                    images[L] = (b["Kfr_" + L], b["Lfr_" + L])
                if q_batch:
                    if kl_out is not None:
                        kls = [kl_out[0:1], kl_out[1:2]]
                    else:   # prediction: the images are wanted, the KL values are not
                        if "kl_scratch" not in b:
                            b["kl_scratch"] = torch.empty(2, dtype=torch.float64, device=X.device)
                        kls = [b["kl_scratch"][0:1], b["kl_scratch"][1:2]]
                    if "qs_ws" not in b:
                        M, K = pf.q_mu.shape
                        b["qs_ws"] = torch.empty(2 * ops._lib.load().mgp_qsqrt_workspace_bytes(M, K),
                                                 dtype=torch.uint8, device=X.device)
                    with _Stage(timing, "split_tri"):
                        ops.qsqrt_images_kl_f16_batch([pf.q_mu, pa.q_mu], [pf.q_sqrt, pa.q_sqrt],
                                                      [b["Lfr_f"], b["Lfr_a"]], kls, workspace=b["qs_ws"])
                elif kl_out is not None:
                    with _Stage(timing, "gauss_kl"):
                        self.pred_layer.prior_kl(out=kl_out[0:1])
                        self.assign_layer.prior_kl(out=kl_out[1:2])
                b["cprep_done"] = False
                if train and _COND_PREP and fmt == "f16" and "cprep_a" in b:
                    # the backward's q_sqrt-only launches, on the forward's L_k image bounds
                    with _Stage(timing, "split_tri"):
                        for L, layer in layers:
                            ops.conditional_backward_prep(
                                layer.q_sqrt, ops.image_bound(b["Lfr_" + L], layer.num_inducing,
                                                              K=layer.num_latent_gps), out=b["cprep_" + L])
                    b["cprep_done"] = True
            if sched == "serial":
                side_work()
            else:
                side.wait_event(prep)   # after Kuu's build (and so after everything before K3 on main)
                with torch.cuda.stream(side):
                    side_work()
                main.wait_stream(side)

            def kuf_late(L):   # a K1 kept off the chain's window (schedules k1a_late, k1_main, serial)
                layer = self.pred_layer if L == "f" else self.assign_layer
                with _Stage(timing, "rbf_kuf"):
                    ops.rbf_kuf_x6(layer.kernel._x(X), layer.Z, layer.kernel.variance, layer.kernel.lengthscales,
                                   out=b["Kfr_" + L], fmt=fmt)
        LinvT = {"f": LinvT_f, "a": LinvT_a}
        bufs = {L: {"Kuf": b["Kuf_" + L], "A": b["A_" + L], "stats": b["stats_" + L],
                    "fmean": b["mu_" + L], "fvar": b["var_" + L], "ws_expert": b["ws_expert"],
                    "Afr": b.get("Afr_" + L, b.get("Afr")), "Tfr": b.get("Tfr_" + L, b.get("Tfr")),
                    "A32": b.get("A32_" + L),
                    "c_out": (b["Cfr_" + L], b["colmax_" + L]) if "Cfr_" + L in b else None} for L, _ in layers}
        if b["x6"] and "Tfr_a" in b:
            # both layers' K4 then both K5 in stream order on the main stream: the
            # matrix-core kernels fill the chip alone, and a cross-stream hand-off
            # costs 10-25 us of idle GPU per wait (measured)
            pf, pa = self.pred_layer, self.assign_layer
            k1a_ev = None

            def side_kuf_a():   # the assign layer's K1 on the side stream from here on
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    kuf_late("a")
                ev = torch.cuda.Event()
                ev.record(side)
                return ev
            if sched == "k1a_late":          # beside the pred layer's K4
                k1a_ev = side_kuf_a()
            elif sched in ("k1_main", "serial"):
                kuf_late("f")
                kuf_late("a")
            bf, ba = bufs["f"], bufs["a"]
            # both layers' K4 in one launch (mgp_trsm_stats_f16_batch, bit-identical to
            # two): one kernel tail and dispatch-round boundary fewer (~25 us, measured)
            batched = (_K4_BATCHED and sched in ("k1_in_k3", "overlap", "k1_main", "serial") and fmt == "f16"
                       and expert_cross() == "f16"
                       and pf.num_inducing == pa.num_inducing and pf.num_latent_gps == pa.num_latent_gps
                       and all(x.get("Afr") is not None and x.get("stats") is not None for x in (bf, ba))
                       and bf["Afr"].data_ptr() != ba["Afr"].data_ptr()
                       and (bf.get("A32") is None) == (ba.get("A32") is None))
            self.layers_per_launch = 2 if batched else 1   # K4 / K5 launches cover this many layers
            if batched:
                with _Stage(timing, "trsm_stats"):
                    (Afr_f, st_f), (Afr_a, st_a) = ops.trsm_stats_f16_batch(
                        [Tfr["f"], Tfr["a"]], [images["f"][0], images["a"][0]], [pf.q_mu, pa.q_mu],
                        pf.num_inducing, N, [bf["Afr"], ba["Afr"]], [bf["stats"], ba["stats"]],
                        [pf.kernel.variance, pa.kernel.variance],
                        As=[bf["A32"], ba["A32"]] if bf.get("A32") is not None else None)
            else:
                Afr_f, st_f = pf.x6_trsm(N, LinvT["f"], images["f"][0], bf, timing, fmt, Tfr=Tfr["f"])
            if sched == "k1a_k5":            # beside the pred layer's K5
                k1a_ev = side_kuf_a()
                pf.x6_expert(N, Afr_f, images["f"][1], st_f, bufs["f"], timing, fmt, colmax_ready=_COLMAX_SIDE)
            if k1a_ev is not None:
                main.wait_event(k1a_ev)
            if not batched:
                Afr_a, st_a = pa.x6_trsm(N, LinvT["a"], images["a"][0], ba, timing, fmt, Tfr=Tfr["a"])
            if batched and "ws_expert2" in b and (bf.get("c_out") is None) == (ba.get("c_out") is None):
                # both layers' K5 in one launch too (mgp_expert_conditional_f16_batch, bit-identical)
                with _Stage(timing, "expert_cond"):
                    c_outs = None
                    if bf.get("c_out") is not None and ba.get("c_out") is not None:
                        c_outs = [bf["c_out"], ba["c_out"]]   # bounds from the side stream's colnorm_max
                        if not _COLMAX_SIDE:
                            ops.colnorm_max(pf.q_sqrt, out=bf["c_out"][1])
                            ops.colnorm_max(pa.q_sqrt, out=ba["c_out"][1])
                    ops.expert_conditional_f16_batch(
                        [Afr_f, Afr_a], [images["f"][1], images["a"][1]], [st_f, st_a],
                        [pf.kernel.variance, pa.kernel.variance], pf.num_inducing, N, pf.num_latent_gps,
                        [bf["fmean"], ba["fmean"]], [bf["fvar"], ba["fvar"]], [b["ws_expert"], b["ws_expert2"]],
                        c_outs=c_outs)
            else:
                if sched != "k1a_k5":
                    pf.x6_expert(N, Afr_f, images["f"][1], st_f, bufs["f"], timing, fmt, colmax_ready=_COLMAX_SIDE)
                pa.x6_expert(N, Afr_a, images["a"][1], st_a, bufs["a"], timing, fmt, colmax_ready=_COLMAX_SIDE)
        else:
            for L, layer in layers:
                if L in late:
                    kuf_late(L)
                layer.conditional_kn(X, LinvT[L], bufs=bufs[L], timing=timing, images=images.get(L), fmt=fmt)
        if kl_out is not None and not b["x6"]:
            with _Stage(timing, "gauss_kl"):
                self.pred_layer.prior_kl(out=kl_out[0:1])
                self.assign_layer.prior_kl(out=kl_out[1:2])
        return b["mu_f"], b["var_f"], b["mu_a"], b["var_a"]

    def _assign_lik_var(self):
        return None  # SMGPModified: the assignment likelihood's variances

    def next_seed(self):
        """Fresh Philox key per evaluation (TF's stateful RNG advances per call)."""
        self._draws += 1
        return _splitmix64(self.seed * 0x100000001B3 + self._draws)

    # ------------------------------------------------------------------ reference methods
    def W_dist(self, Xt, noise_z=None, seed=None, n_offset=0, tiled=None):
        """SMGP.W_dist (models.py:55-61): the assign layer's marginals, reparameterised
        with z ~ N(0, 1) [S, N, K] (utils.py:26-27) into logits [S * N, K], as a
        RelaxedOneHotCategorical(1e-2).  noise_z: explicit normals [S, N, K]; else
        Philox with `seed` (a fresh key per call when None), K6's z stream.  tiled:
        SVGPModified._marginals_kn's switch for materialised S-tiled inputs."""
        fm, fv, S, N, stride, _ = self.assign_layer._marginals_kn(Xt, tiled=tiled)
        if seed is None and noise_z is None:
            seed = self.next_seed()
        logits = ops.assign_logits(fm, fv, S, N, stride, noise_z=noise_z, seed=seed or 0, n_offset=n_offset)
        return RelaxedOneHotCategorical(TAU, logits.reshape(S * N, self.K), (S, N), seed=seed, n_offset=n_offset,
                                        model=self)

    def E_log_p_Y(self, Xt, Y, W_SND, tiled=None):
        """SMGP.E_log_p_Y (models.py:63-67): logsumexp_S(sum_K W ve) - log S -> [N]
        (device float32), ve the pred likelihood's variational expectation."""
        fm, fv, S, N, stride, _ = self.pred_layer._marginals_kn(Xt, tiled=tiled)
        Yd = _to_dev(Y, self.device).reshape(-1).contiguous()
        W = _to_dev(W_SND, self.device)
        mc = self._mc_eps()
        lik_var = None if mc is not None else self.likelihood.likelihood.variance.reshape(-1)
        extra = {}
        if self._assign_lik_var() is not None:   # SMGPModified.E_log_p_Y (models.py:112-123)
            fa, va, Sa, Na, stride_a, _ = self.assign_layer._marginals_kn(Xt, tiled=tiled)
            if (Sa, Na, stride_a) != (S, N, stride):
                raise ValueError("the two layers' marginals disagree in shape")
            extra = dict(mu_a=fa, var_a=va, assign_lik_var=self._assign_lik_var())
        return ops.e_log_p_y(fm, fv, Yd, lik_var, W, S, N, stride, multiclass_eps=mc, **extra)

    @property
    def trainable_variables(self):
        """GPflow Module.trainable_variables (utils/training_utils.py:10): the device
        tensors of trainable_parameters(), in its order.  These hold the CONSTRAINED
        values (what every kernel reads); GPflow's tf.Variables hold the unconstrained
        ones (softplus^-1 for positive parameters).  run_adam / AdamTF keep the
        unconstrained shadows themselves; a custom loop gets GPflow's semantics from
        unconstrained_variables(), elbo_and_grad(..., unconstrained=True) and
        assign_unconstrained() (tests/test_gpu_api.py)."""
        return tuple(t for _, t, _ in self.trainable_parameters())

    # ------------------------------------------------------------------ ELBO
    def _build_likelihood(self, X, Y, noise=None, seed=None, n_offset=0, n_total=None,
                          process_group=None, return64=False, timing=None):
        """ELBO (models.py:69-79) as a 0-d float32 device tensor.

        noise: optional explicit (z, u) [S, N, K] device tensors (parity mode);
        otherwise in-kernel Philox keyed by (seed, global n, s, k).
        n_offset / n_total / process_group: data-parallel sharding over N (each
        rank passes its shard; one all-reduce of the data-term sum)."""
        X = self.pred_layer.kernel._x(X)
        N = X.shape[0]
        Yd = _to_dev(Y, self.device).reshape(-1).contiguous()
        if Yd.numel() != N:
            raise ValueError("X and Y must have the same number of rows")
        b = self._buffers(N)
        kl = b["kl"]
        mu_f, var_f, mu_a, var_a = self.conditionals(X, timing=timing, kl_out=kl)
        mc = self._mc_eps()
        lik_var = None if mc is not None else self.likelihood.likelihood.variance.reshape(-1)
        if seed is None and noise is None:
            seed = self.next_seed()
        with _Stage(timing, "elbo_terms"):
            ops.elbo_terms(mu_f, var_f, mu_a, var_a, Yd, lik_var, self.num_samples, TAU,
                           noise=noise, seed=seed or 0, n_offset=n_offset, out=b["data_sum"],
                           assign_lik_var=self._assign_lik_var(), multiclass_eps=mc)
        if process_group is not None:
            import torch.distributed as dist
            with _Stage(timing, "allreduce"):
                dist.all_reduce(b["data_sum"], op=dist.ReduceOp.SUM, group=process_group)
        n_batch = n_total if n_total is not None else N
        num_data = self.num_data if self.num_data is not None else n_batch
        # a fresh tensor per call (the reference returns a new value each time), written
        # by the combine kernel itself (no copy launch behind it)
        e32 = torch.empty((), dtype=torch.float32, device=self.device)
        e64 = torch.empty((), dtype=torch.float64, device=self.device)
        ops.elbo_combine(b["data_sum"], kl[0:1], kl[1:2], n_batch, num_data, out=e32, out64=e64)
        return e64 if return64 else e32

    # ------------------------------------------------------------------ training
    def trainable_parameters(self):
        """[(name, tensor, transform)] of every trainable variable (Z, q_mu,
        q_sqrt (lower triangle), kernel variance / lengthscales (softplus) of both layers,
        and the shared Gaussian likelihood variance (softplus))."""
        ps = []
        for name, layer in (("pred", self.pred_layer), ("assign", self.assign_layer)):
            ps += [(name + ".Z", layer.Z, "free"), (name + ".q_mu", layer.q_mu, "free"),
                   (name + ".q_sqrt", layer.q_sqrt, "free"),
                   (name + ".variance", layer.kernel.variance, "positive"),
                   (name + ".lengthscales", layer.kernel.lengthscales, "positive")]
        if self._mc_eps() is None:  # MultiClass / RobustMax: no trainable likelihood parameter
            ps.append(("lik_variance", self.likelihood.likelihood.variance, "positive"))
        if self._assign_lik_var() is not None:
            ps.append(("assign_lik_variance", self.assign_likelihood.likelihood.variance, "positive"))
        return ps

    def unconstrained_variables(self):
        """{name: device tensor} of the unconstrained values GPflow's trainable_variables
        hold (utils/training_utils.py:10 differentiates w.r.t. these): free parameters as
        they are, positive ones as u = softplus^-1(theta) (gpflow.utilities.positive(),
        float64 inverse, then float32; the value theta = softplus(u) reproduces theta)."""
        out = {}
        for name, t, kind in self.trainable_parameters():
            if kind == "positive":
                th = t.detach().double()
                out[name] = torch.where(th > 20, th, torch.log(torch.expm1(th))).float()
            else:
                out[name] = t.detach().clone()
        return out

    def assign_unconstrained(self, values):
        """Set parameters from unconstrained values (dict name -> tensor, e.g. after a
        custom optimiser step on unconstrained_variables()): theta = softplus(u) for
        positive parameters, in place, so every kernel reads the new state."""
        for name, t, kind in self.trainable_parameters():
            if name not in values:
                continue
            v = values[name].to(device=t.device, dtype=torch.float32).reshape(t.shape)
            t.copy_(torch.nn.functional.softplus(v.double()).float() if kind == "positive" else v)

    def _tail_batchable(self):
        """Both layers' Cholesky / RBF backward can share launches: same M, D and
        lengthscale count (mgp_chol_backward_batch, mgp_rbf_backward_batch)."""
        f, a = self.pred_layer, self.assign_layer
        return (f.Z.shape == a.Z.shape and f.kernel.lengthscales.numel() == a.kernel.lengthscales.numel()
                and f.Z.stride() == a.Z.stride())

    def elbo_and_grad(self, X, Y, noise=None, seed=None, n_offset=0, n_total=None, process_group=None,
                      timing=None, unconstrained=False):
        """ELBO (0-d float32) and its gradient w.r.t. every constrained parameter of
        trainable_parameters() (dict name -> device tensor; unconstrained=True: w.r.t.
        the unconstrained values of unconstrained_variables(), GPflow's
        trainable_variables, by the softplus chain rule), i.e. the GradientTape pass
        of run_adam's optimisation step (training_utils.py:10) on the HIP kernels:
        K6 backward -> per layer conditional backward (x6) -> Cholesky backward -> RBF
        backward (Kuf and Kuu) -> + KL.  Data-parallel: one all-reduce of the
        data-term gradients per step (the KL part is added after it)."""
        X = self.pred_layer.kernel._x(X)
        N = X.shape[0]
        Yd = _to_dev(Y, self.device).reshape(-1).contiguous()
        b = self._buffers(N, train=True)
        kl = b["kl"]
        mu_f, var_f, mu_a, var_a = self.conditionals(X, timing=timing, kl_out=kl, train=True)
        mc = self._mc_eps()
        lik_var = None if mc is not None else self.likelihood.likelihood.variance.reshape(-1)
        alv = self._assign_lik_var()
        if seed is None and noise is None:
            seed = self.next_seed()
        with _Stage(timing, "elbo_terms"):
            ops.elbo_terms(mu_f, var_f, mu_a, var_a, Yd, lik_var, self.num_samples, TAU, noise=noise,
                           seed=seed or 0, n_offset=n_offset, out=b["data_sum"], assign_lik_var=alv,
                           multiclass_eps=mc)
        n_batch = n_total if n_total is not None else N
        with _Stage(timing, "elbo_terms_bwd"):
            G, glv, glva = ops.elbo_terms_backward(mu_f, var_f, mu_a, var_a, Yd, lik_var, self.num_samples, TAU,
                                                   noise=noise, seed=seed or 0, n_offset=n_offset,
                                                   scale=1.0 / n_batch, assign_lik_var=alv, G=b["G"],
                                                   multiclass_eps=mc)
        grads = {"lik_variance": glv} if mc is None else {}
        if alv is not None:
            grads["assign_lik_variance"] = glva

        def cond_backward(L, layer, gi, ws):
            M = layer.num_inducing
            with _Stage(timing, "conditional_bwd"):
                cimg = None
                if "Cfr_" + L in b:  # the forward's C_k images (mgp_conditional_backward_f16c)
                    cimg = (b["Cfr_" + L], b["colmax_" + L],
                            ops.image_bound(b["Lfr_" + L], M, K=layer.num_latent_gps))
                prep = b["cprep_" + L] if cimg is not None and b.get("cprep_done") else None
                tb = ops.image_bound(b["Tfr_" + L], M, K=1) if prep is not None and b.get("lt_bounded") and _T_BOUND else None
                return ops.conditional_backward_x6(b["Afr_" + L], b["A32_" + L], layer.q_sqrt,
                                                   layer.q_mu, b["LinvT_" + L], G[gi], G[gi + 1], M, N,
                                                   workspace=ws, fmt=forward_image_format(True),
                                                   c_images=cimg, prep=prep, t_bound=tb)

        def tail_backward(L, name, layer, g):
            with _Stage(timing, "chol_bwd"):
                gKuu = ops.chol_backward(b["L_" + L], b["LinvT_" + L], g["g_Lm"])
            with _Stage(timing, "rbf_bwd"):
                k = layer.kernel
                gZ, gvar, gls = ops.rbf_backward(X, layer.Z, k.variance, k.lengthscales, g["g_Kuf"],
                                                 accumulate=True, g_var=g["g_var"],
                                                 gZ=torch.zeros_like(layer.Z),
                                                 g_ls=torch.zeros(k.lengthscales.numel(), dtype=torch.float64,
                                                                  device=self.device))
                ops.rbf_backward(layer.Z, layer.Z, k.variance, k.lengthscales, gKuu, symmetric=True,
                                 accumulate=True, gZ=gZ, g_var=gvar, g_ls=gls)
            return {name + ".Z": gZ, name + ".variance": gvar, name + ".lengthscales": gls,
                    name + ".q_mu": g["g_q_mu"], name + ".q_sqrt": g["g_q_sqrt"]}

        def tail_backward_batch(order, gs):
            with _Stage(timing, "chol_bwd"):
                gKuus = ops.chol_backward_batch([b["L_" + L] for L, *_ in order], [b["LinvT_" + L] for L, *_ in order],
                                                [g["g_Lm"] for g in gs])
            with _Stage(timing, "rbf_bwd"):
                layers = [layer for _, _, layer, _ in order]
                # gZ / g_ls written by the finish (accumulate 2: no zero fills), g_var added
                # to the conditional backward's part
                alloc = torch.empty if _RBF_NO_FILL else torch.zeros
                gZs = [alloc(layer.Z.shape, dtype=layer.Z.dtype, device=self.device) for layer in layers]
                glss = [alloc(layer.kernel.lengthscales.numel(), dtype=torch.float64, device=self.device)
                        for layer in layers]
                ops.rbf_backward_batch(X, [layer.Z for layer in layers], [layer.kernel.variance for layer in layers],
                                       [layer.kernel.lengthscales for layer in layers], [g["g_Kuf"] for g in gs],
                                       gKuus, gZs, [g["g_var"] for g in gs], glss,
                                       accumulate=2 if _RBF_NO_FILL else 1)
            return [{name + ".Z": gZ, name + ".variance": g["g_var"], name + ".lengthscales": gls,
                     name + ".q_mu": g["g_q_mu"], name + ".q_sqrt": g["g_q_sqrt"]}
                    for (_, name, _, _), g, gZ, gls in zip(order, gs, gZs, glss)]

        pending = []

        def reduce_bucket(layer_grads):
            if process_group is not None:
                # one bucket per layer (the first also carries the data-term sum and the
                # likelihood gradients); the pred layer's is in flight while the assign
                # layer's backward still runs
                from .distributed import allreduce_gradients_async
                bucket = list(layer_grads.values())
                if not pending:
                    bucket = [b["data_sum"]] + list(grads.values()) + bucket
                pending.append(allreduce_gradients_async(bucket, group=process_group))

        # the two layers in order on this stream (a side stream for one layer's Cholesky /
        # RBF backward beside the other's conditional backward measured slower: the
        # matrix-core kernel starves the small ones, DESIGN.md round-4 results); with
        # matching shapes both layers' Cholesky and RBF backward run as one batch each
        order = (("f", "pred", self.pred_layer, 0), ("a", "assign", self.assign_layer, 2))
        if _TAIL_BATCH and self._tail_batchable():
            gs = [cond_backward(L, layer, gi, b["ws_cbwd"]) for L, _, layer, gi in order]
            for layer_grads in tail_backward_batch(order, gs):
                reduce_bucket(layer_grads)
                grads.update(layer_grads)
        else:
            for L, name, layer, gi in order:
                layer_grads = tail_backward(L, name, layer, cond_backward(L, layer, gi, b["ws_cbwd"]))
                reduce_bucket(layer_grads)
                grads.update(layer_grads)
        if process_group is not None:
            with _Stage(timing, "allreduce"):
                for pb in pending:
                    pb.wait()
        num_data = self.num_data if self.num_data is not None else n_batch
        for name, layer in (("pred", self.pred_layer), ("assign", self.assign_layer)):
            ops.kl_grad(layer.q_mu, layer.q_sqrt, num_data, grads[name + ".q_mu"], grads[name + ".q_sqrt"])
        e32 = torch.empty((), dtype=torch.float32, device=self.device)   # fresh per call, no copy launch
        ops.elbo_combine(b["data_sum"], kl[0:1], kl[1:2], n_batch, num_data, out=e32, out64=b["elbo64"])
        if unconstrained:   # d/du = d/dtheta * softplus'(u) = d/dtheta * (1 - exp(-theta)) for positive ones
            for name, t, kind in self.trainable_parameters():
                if kind == "positive":
                    grads[name] = grads[name] * (-torch.expm1(-t.double())).float()
        return e32, grads

    def training_loss_closure(self, data_iter, compile=True):
        """GPflow ExternalDataTrainingLossMixin.training_loss_closure: () -> -ELBO on the next batch."""
        def closure():
            X, Y = next(data_iter)
            return self.training_loss((X, Y))
        return closure

    def elbo(self, data, **kw):
        X, Y = data
        return self._build_likelihood(X, Y, **kw)

    def _training_loss(self, data):
        """models.py:81-83."""
        X, Y = data
        return -self._build_likelihood(X, Y)

    def training_loss(self, data):
        return self._training_loss(data)

    # ------------------------------------------------------------------ predictions
    def predict_assign(self, Xnew, S=1):
        """models.py:85-89: softmax_K(mean_S mu_a) -> [N, K] host array (HostArray, float64)."""
        asg = self.predict_assign_device(Xnew, S)
        self.check_linalg(self.assign_layer._last_info)
        return _host(asg)

    def predict_assign_device(self, Xnew, S=1):
        """predict_assign as a float32 device tensor [N, K]."""
        X = self.assign_layer.kernel._x(Xnew)
        am, _ = self.assign_layer.conditional_kn(X)
        _, _, asg = ops.predict_epilogue(None, None, am, None, want_y=False, want_assign=True)
        return asg

    def predict_samples(self, Xnew, S=1, noise=None, seed=None):
        """models.py:91-103 -> samples_y, samples_f [S, N, 1] host arrays (HostArray, float64)."""
        sy, sf = self.predict_samples_device(Xnew, S, noise=noise, seed=seed)
        self.check_linalg()
        return _host(sy), _host(sf)

    def predict_samples_device(self, Xnew, S=1, noise=None, seed=None):
        """predict_samples as float32 device tensors [S, N, 1]."""
        X = self.pred_layer.kernel._x(Xnew)
        mu_f, var_f, mu_a, var_a = self.conditionals(X)
        if seed is None and noise is None:
            seed = self.next_seed()
        mc = self._mc_eps()
        sy, sf = ops.predict_samples(mu_f, var_f, mu_a, var_a,
                                     None if mc is not None else self.likelihood.likelihood.variance.reshape(-1),
                                     S, TAU, noise=noise, seed=seed or 0, multiclass_eps=mc)
        return sy[..., None], sf[..., None]


class SMGPModified(SMGP):
    """SMGP with a second (assignment) Gaussian likelihood on the assign layer
    (models.py:106-123): E_log_p_Y = lse_S(sum_k W ve_a) + lse_S(sum_k W ve_f) - 2 log S,
    both weighted by the same W.  The assign-layer conditional feeds both W and
    ve_a (the reference computes it twice, :113 and in W_dist); the data term is
    the MOD variant of K6 (mgp_elbo_terms_modified)."""

    def __init__(self, likelihood, assign_likelihood, pred_layer, assign_layer, K=3, num_samples=1,
                 num_data=None, seed=0):
        SMGP.__init__(self, likelihood, pred_layer, assign_layer, K, num_samples, num_data, seed)
        self.assign_likelihood = BroadcastingLikelihood(assign_likelihood)

    def _assign_lik_var(self):
        return self.assign_likelihood.likelihood.variance.reshape(-1)
