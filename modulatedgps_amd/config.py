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
_CFG = {"jitter": 1e-6, "device": None, "conditional": os.environ.get("MGP_CONDITIONAL", "x6"),
        "expert_planes": int(os.environ.get("MGP_K5_PLANES", "3"))}


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
