"""Counter-based Philox4x32-10 noise, numpy restatement (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import anything under ``oracle/``.  The product path never does.

Why this exists: the reference draws its Monte-Carlo noise from TensorFlow's
stateful RNG (``tf.random.normal`` at ``MixtureGPs/models.py:57`` and TFP's
``samplers.uniform`` inside ``RelaxedOneHotCategorical.sample`` at
``MixtureGPs/models.py:60,73``).  That stream cannot be reproduced without TF,
so the MI355X build draws its noise in-kernel from Philox4x32-10 keyed by the
GLOBAL (sample s, data point n, expert k) index, which makes results invariant
to how N is sharded over GPUs.  This module is the bit-exact host statement of
that stream (the uint32 words are bit-exact; the float transforms are computed
in float64 here and in float32 on the GPU).

Algorithm: Salmon et al., "Parallel random numbers: as easy as 1, 2, 3"
(SC'11), Philox4x32 with 10 rounds, constants from the Random123 distribution.

Stream layout (must match ``modulatedgps_amd/csrc/mgp_philox.hpp``):
  key      = (seed & 0xffffffff, seed >> 32)
  counter  = (n, s, k >> 2, stream)      stream 0 -> normals z, 1 -> uniforms u,
                                         stream 2 -> normals of predict_samples' y/f draws
  word     = k & 3
  uniform  = ((w >> 9) + 0.5) * 2**-23               in (0, 1), never 0 or 1
  normal   = Box-Muller on the (w0, w1) / (w2, w3) word pairs of the z block:
             r = sqrt(-2 log u0), z0 = r cos(2 pi u1), z1 = r sin(2 pi u1)
"""
import numpy as np

PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = np.uint32(0x9E3779B9)
PHILOX_W1 = np.uint32(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: uint32 array [..., 2] (broadcastable).

    Returns uint32 array [..., 4].
    """
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    c0, c1, c2, c3 = (ctr[..., i].astype(np.uint32) for i in range(4))
    k0 = np.broadcast_to(key[..., 0], c0.shape).astype(np.uint32)
    k1 = np.broadcast_to(key[..., 1], c0.shape).astype(np.uint32)
    for _ in range(10):
        p0 = PHILOX_M0 * c0.astype(np.uint64)
        p1 = PHILOX_M1 * c2.astype(np.uint64)
        hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
        lo0 = (p0 & _MASK32).astype(np.uint32)
        hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
        lo1 = (p1 & _MASK32).astype(np.uint32)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        with np.errstate(over="ignore"):
            k0 = (k0 + PHILOX_W0).astype(np.uint32)
            k1 = (k1 + PHILOX_W1).astype(np.uint32)
    return np.stack([c0, c1, c2, c3], axis=-1)


def _key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)


def u01(words):
    """uint32 -> float in (0,1): ((w >> 9) + 0.5) * 2^-23 (exact in fp32 and fp64)."""
    w = np.asarray(words, dtype=np.uint32)
    return ((w >> np.uint32(9)).astype(np.float64) + 0.5) * (2.0 ** -23)


def _blocks(seed, S, n_global, K, stream):
    """Philox output words for every (s, n, k-block): shape [S, N, ceil(K/4), 4]."""
    n_global = np.asarray(n_global, dtype=np.uint64)
    nb = (K + 3) // 4
    s = np.arange(S, dtype=np.uint32)[:, None, None]
    n = (n_global & _MASK32).astype(np.uint32)[None, :, None]
    b = np.arange(nb, dtype=np.uint32)[None, None, :]
    shape = (S, n_global.shape[0], nb)
    ctr = np.stack([np.broadcast_to(n, shape), np.broadcast_to(s, shape),
                    np.broadcast_to(b, shape),
                    np.full(shape, stream, dtype=np.uint32)], axis=-1)
    return philox4x32_10(ctr, _key(seed))


def noise_uniform(seed, S, n_global, K):
    """u[s, n, k] in (0,1) for the Gumbel noise of A.5 (float64)."""
    w = _blocks(seed, S, n_global, K, 1)
    u = u01(w).reshape(S, len(n_global), -1)
    return u[:, :, :K]


def noise_normal(seed, S, n_global, K, stream=0):
    """z[s, n, k] ~ N(0,1) via Box-Muller on the stream words (float64)."""
    w = _blocks(seed, S, n_global, K, stream)
    u = u01(w)                                         # [S, N, nb, 4]
    r0 = np.sqrt(-2.0 * np.log(u[..., 0]))
    r1 = np.sqrt(-2.0 * np.log(u[..., 2]))
    t0 = 2.0 * np.pi * u[..., 1]
    t1 = 2.0 * np.pi * u[..., 3]
    z = np.stack([r0 * np.cos(t0), r0 * np.sin(t0), r1 * np.cos(t1), r1 * np.sin(t1)], axis=-1)
    z = z.reshape(S, len(n_global), -1)
    return z[:, :, :K]
