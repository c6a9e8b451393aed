"""Global configuration mirroring the GPflow globals the reference relies on
(MixtureGPs/models.py:16-17: default_float / default_jitter), plus the device.

The compute dtype of this build is float32 (the MI355X path); the reference's
float64 semantics are the parity target (tolerances in tests/)."""
import os

import torch

# conditional: "x6" = K5 on split-bf16 fragment images (f32-accurate, bf16 MFMA),
#              "f32" = K5 on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32).
# expert_planes (x6 mode): bf16 planes per operand in K5 -- 3 (default: six
#              products, f32-accurate), 2 (three products, ~16-bit operands) or
#              1 (bf16 operands): BASELINE config 5's "bf16 mixed" (K1-K4 stay x6).
# expert_format (x6 mode, forward evaluations): the A and tril(q_sqrt) images K5
#              reads -- "f16" (default: split-f16, three f16 products at 22-bit
#              operands; csrc/mgp_common.hpp) or "x6" (split-bf16, six bf16
#              products).  Both measure the same error against the float64 oracle
#              (tests/test_gpu_f16.py: 1.0e-7 normwise on K5's term, 7.3e-7 on fvar
#              at c3 shapes -- the f32 inputs' own rounding); f16 is half the MFMA
#              work.  The training step follows it (A's image, S_k A in the
#              backward); the reduced-plane modes use "x6".
_CFG = {"jitter": 1e-6, "device": None, "conditional": "x6", "expert_planes": 3, "expert_format": "f16",
        "expert_cross": "f16", "step_schedule": "k1_in_k3"}
# expert_cross (f16 images): the precision of K5's two cross-term products
#              a_hi b_lo + a_lo b_hi -- "f16" (three f16 products) or "f8" (one
#              e4m3 MFMA per two k-steps for both, mgp_expert_conditional_f16x8:
#              the cross terms are 2^-11 of the leading product, so their 3-bit
#              mantissas cost ~2^-15 relative; tests/test_gpu_f16.py measures it).


def default_jitter():
    return _CFG["jitter"]


def set_default_jitter(v):
    _CFG["jitter"] = float(v)


def default_float():
    return torch.float32


def default_device():
    if _CFG["device"] is not None:
        return _CFG["device"]
    if not torch.cuda.is_available():
        raise RuntimeError("modulatedgps_amd needs a HIP device (MI355X); none is visible")
    return torch.device("cuda", torch.cuda.current_device())


def set_default_device(dev):
    _CFG["device"] = torch.device(dev)


def conditional_mode():
    return _CFG["conditional"]


def set_conditional_mode(mode):
    if mode not in ("x6", "f32"):
        raise ValueError("conditional mode must be 'x6' or 'f32'")
    _CFG["conditional"] = mode


def expert_planes():
    return _CFG["expert_planes"]


def set_expert_planes(planes):
    if planes not in (1, 2, 3):
        raise ValueError("expert_planes must be 1, 2 or 3")
    _CFG["expert_planes"] = int(planes)


def expert_format():
    return _CFG["expert_format"]


def set_expert_format(fmt):
    if fmt not in ("x6", "f16"):
        raise ValueError("expert_format must be 'x6' or 'f16'")
    _CFG["expert_format"] = fmt


def expert_cross():
    return _CFG["expert_cross"]


def set_expert_cross(cross):
    if cross not in ("f16", "f8"):
        raise ValueError("expert_cross must be 'f16' or 'f8'")
    _CFG["expert_cross"] = cross


# step_schedule (x6 mode): where the Cholesky-independent work of an ELBO step runs
#              relative to the latency-bound K3 chain (host-side launch order only;
#              every schedule computes the same bits):
#   "k1_in_k3" (default since round 5) both layers' K1 run inside K3's step launches, on
#              extra workgroups that take the CUs the latency-bound chain leaves idle
#              (mgp_kuu_potrf_trtri_kuf: the same image blocks, bit-identical); the
#              tril(q_sqrt) images and the KL on the side stream as in "overlap".  Beside
#              the chain on a side stream, K1's 8192 workgroups held the CUs that the
#              next step launch's workgroups waited for (32-41 us gaps, round 4 stamps);
#              with batched K3 only (equal M for both layers), else as "overlap";
#   "overlap"  K1 and the tril(q_sqrt) images of both layers and the KL on a side
#              stream beside K3 (round 1-4 default);
#   "k1a_late" the assign layer's K1 on the side stream after K3, beside the pred
#              layer's K4 (one K1 beside the chain instead of two);
#   "k1a_k5"   as k1a_late, but the layers run K4, K5 of the pred layer before the
#              assign layer's K4, so that K1 runs beside the MFMA-bound K5;
#   "k1_main"  both K1 on the main stream after K3 (only the small images and
#              the KL beside the chain);
#   "serial"   everything on the main stream, K3 alone on the chip.
STEP_SCHEDULES = ("k1_in_k3", "overlap", "k1a_late", "k1a_k5", "k1_main", "serial")


def step_schedule():
    return _CFG["step_schedule"]


def set_step_schedule(name):
    if name not in STEP_SCHEDULES:
        raise ValueError(f"step schedule must be one of {STEP_SCHEDULES}")
    _CFG["step_schedule"] = name


def forward_image_format(train=False):
    """Image format of the K1 -> K4 -> K5 chain (and of the training step's A
    image): expert_format() at full planes, "x6" for the reduced-plane modes."""
    if expert_planes() != 3:
        return "x6"
    return expert_format()


def _from_env():
    """Environment overrides, validated by the setters (a bad value raises at import)."""
    env = os.environ
    if "MGP_CONDITIONAL" in env:
        set_conditional_mode(env["MGP_CONDITIONAL"])
    if "MGP_K5_PLANES" in env:
        try:
            planes = int(env["MGP_K5_PLANES"])
        except ValueError:
            raise ValueError(f"MGP_K5_PLANES={env['MGP_K5_PLANES']!r} is not 1, 2 or 3") from None
        set_expert_planes(planes)
    if "MGP_K5_FORMAT" in env:
        set_expert_format(env["MGP_K5_FORMAT"])
    if "MGP_K5_CROSS" in env:
        set_expert_cross(env["MGP_K5_CROSS"])
    if "MGP_STEP_SCHEDULE" in env:
        set_step_schedule(env["MGP_STEP_SCHEDULE"])


_from_env()
