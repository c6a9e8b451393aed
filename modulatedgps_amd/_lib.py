"""ctypes binding of libmgp_hip.so (the C-ABI declared in include/mgp_hip.h).

There is deliberately no fallback: if the HIP library is missing or cannot be
loaded, every op raises ``MGPLibraryError``.  The product path never computes
on the CPU.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MGP_HIP_LIB", os.path.join(_HERE, "libmgp_hip.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "mgp_hip.h")


class MGPLibraryError(RuntimeError):
    """libmgp_hip.so is missing or could not be loaded."""


class MGPError(RuntimeError):
    """A libmgp_hip call returned a non-zero status."""

    def __init__(self, fn, status, msg):
        super().__init__(f"{fn} failed with status {status}: {msg}")
        self.status = status


class MGPLinAlgError(MGPError):
    """Cholesky of Kuu failed (non-positive pivot), like TF's InvalidArgumentError
    raised from base_conditional (MixtureGPs/models.py:141)."""


c_f32p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_u64 = ctypes.c_uint64
c_size = ctypes.c_size_t
c_ptr = ctypes.c_void_p

# name -> (restype, argtypes); must mirror include/mgp_hip.h
SIGNATURES = {
    "mgp_version": (ctypes.c_char_p, []),
    "mgp_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "mgp_rbf_kuf": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr,
                                   c_i32, c_ptr, c_i64, c_ptr]),
    "mgp_rbf_kuu": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i32, ctypes.c_float,
                                   c_ptr, c_i64, c_ptr]),
    "mgp_chol_workspace_bytes": (c_size, [c_i64, c_i32]),
    "mgp_potrf_trtri": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i64, c_i64,
                                       c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_kuu_potrf_trtri": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_ptr,
                                           ctypes.c_float, c_i32, c_ptr, c_ptr, c_i64, c_i64, c_ptr,
                                           c_ptr, c_size, c_ptr]),
    "mgp_kuu_potrf_trtri_ev": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_ptr,
                                           ctypes.c_float, c_i32, c_ptr, c_ptr, c_i64, c_i64, c_ptr,
                                           c_ptr, c_size, c_ptr, c_ptr]),
    "mgp_kuu_potrf_trtri_ex": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_ptr,
                                           ctypes.c_float, c_i32, c_ptr, c_ptr, c_i64, c_i64, c_ptr,
                                           c_ptr, c_size, c_ptr, c_ptr, c_ptr]),
    "mgp_kuu_potrf_trtri_kuf": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_ptr,
                                            ctypes.c_float, c_i32, c_ptr, c_ptr, c_i64, c_i64, c_ptr,
                                            c_ptr, c_size, c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_size,
                                            c_i32, c_ptr]),
    "mgp_stats_tiles": (ctypes.c_int, [c_i64]),
    "mgp_trsm_stats": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i32,
                                      c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "mgp_expert_workspace_bytes": (c_size, [c_i64, c_i64, c_i32]),
    "mgp_expert_conditional_f32": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr,
                                                  c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size,
                                                  c_ptr]),
    # the SURVEY §8(b) front (csrc/front.hip)
    "mgp_workspace_bytes": (c_size, [c_i32, c_i64, c_i64, c_i32]),
    "mgp_rbf_kuu_jitter": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i32, ctypes.c_float,
                                          c_ptr, c_i64, c_ptr]),
    "mgp_potrf_lower": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_trsm_lln": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_expert_conditional": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64,
                                              c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_trsm_stats_x6": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_i64, c_i64, c_ptr, c_i64, c_i32,
                                         c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "mgp_kl_grad": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, ctypes.c_double, c_ptr,
                                   c_i64, c_ptr, c_i64, c_i64, c_ptr]),
    "mgp_adam_step": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_i32, c_i64, c_ptr, c_ptr, c_i64, c_i64, c_i64,
                                     ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, c_i64,
                                     ctypes.c_float, c_ptr]),
    "mgp_adam_step_set": (ctypes.c_int, [c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
                                         c_ptr, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                         c_i64, ctypes.c_float, c_ptr]),
    "mgp_rbf_backward_workspace_bytes": (c_size, [c_i64, c_i64, c_i32]),
    "mgp_rbf_backward": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i32,
                                        c_ptr, c_i64, c_i32, c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_size,
                                        c_ptr]),
    "mgp_rbf_backward_batch_workspace_bytes": (c_size, [c_i64, c_i64, c_i32]),
    "mgp_rbf_backward_batch": (ctypes.c_int, [c_i32, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i32, c_ptr, c_ptr,
                                              c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_ptr, c_i64, c_ptr, c_ptr,
                                              c_ptr, c_size, c_ptr]),
    "mgp_chol_backward_batch": (ctypes.c_int, [c_i32, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_ptr,
                                               c_i64, c_ptr, c_size, c_ptr]),
    "mgp_chol_backward_workspace_bytes": (c_size, [c_i64]),
    "mgp_chol_backward": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr,
                                         c_size, c_ptr]),
    "mgp_gram_workspace_bytes": (c_size, [c_i64, c_i64, c_i64, c_i32]),
    "mgp_gram": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, ctypes.c_float, c_i32, c_ptr,
                                c_i64, c_ptr, c_size, c_ptr]),
    "mgp_gram_x6_workspace_bytes": (c_size, [c_i64, c_i64, c_i64, c_i32, c_i32]),
    "mgp_gram_x6": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64,
                                   c_i32, ctypes.c_float, c_i32, c_ptr, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_gram_f16": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64,
                                    c_i32, ctypes.c_float, c_i32, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr,
                                    c_size, c_ptr]),
    "mgp_rows_f16_ksteps": (c_i64, [c_i64]),
    "mgp_rows_f16_bytes": (c_size, [c_i64, c_i64]),
    "mgp_split_rows_f16": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_gram_f16_rows": (ctypes.c_int, [c_ptr, c_size, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i32,
                                         ctypes.c_float, c_i32, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr,
                                         c_size, c_ptr]),
    "mgp_conditional_backward_workspace_bytes": (c_size, [c_i64, c_i64, c_i32]),
    "mgp_conditional_backward_x6": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                   c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                                   c_i64, c_i64, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64,
                                                   c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_conditional_backward_f16": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                   c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                                   c_i64, c_i64, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64,
                                                   c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_conditional_backward_f16x8": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                   c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                                   c_i64, c_i64, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64,
                                                   c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_conditional_backward_f16c": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                    c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                                    c_i64, c_i64, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64,
                                                    c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr,
                                                    c_size, c_ptr, c_ptr, c_ptr]),
    "mgp_conditional_backward_prep_bytes": (c_size, [c_i64, c_i32]),
    "mgp_conditional_backward_prep_f16c": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_size,
                                                         c_ptr]),
    "mgp_conditional_backward_f16c_prepped": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                            c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_i64,
                                                            c_i64, c_i64, c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64,
                                                            c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr,
                                                            c_size, c_ptr, c_ptr, c_ptr, c_size, c_ptr, c_ptr]),
    "mgp_c_images_bytes": (c_size, [c_i64, c_i64, c_i32]),
    "mgp_colnorm_max": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr]),
    "mgp_expert_conditional_f16c": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                   c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size, c_ptr, c_size,
                                                   c_ptr, c_ptr]),
    "mgp_split_upper_x6": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_rbf_kuf_x6": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i32,
                                      c_ptr, c_size, c_ptr]),
    "mgp_x6_lower_bytes": (c_size, [c_i64, c_i32]),
    "mgp_x6_cols_bytes": (c_size, [c_i64, c_i64]),
    "mgp_split_lower_x6": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_size, c_ptr]),
    "mgp_split_cols_x6": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_expert_x6_workspace_bytes": (c_size, [c_i64, c_i64, c_i32]),
    "mgp_expert_conditional_x6": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                 c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_expert_conditional_planes": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                     c_i64, c_i32, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size,
                                                     c_ptr]),
    "mgp_split_lower_f16": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_size, c_ptr]),
    "mgp_split_cols_f16": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_trsm_stats_x6_f16": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_i64, c_i64, c_ptr, c_i64, c_i32,
                                             c_ptr, c_ptr, c_size, c_ptr, c_i64, c_ptr]),
    "mgp_rbf_kuf_f16": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i32,
                                       c_ptr, c_size, c_ptr]),
    "mgp_split_upper_f16": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_split_upper_f16_bounded": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_split_upper_f16_bounded_batch": (ctypes.c_int, [c_i32, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_x6_bound_ptr": (ctypes.c_void_p, [c_ptr, c_i64, c_i64, c_i32]),
    "mgp_trsm_stats_f16": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_i64, c_i64, c_ptr, c_i64, c_i32,
                                          c_ptr, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "mgp_trsm_stats_f16_batch": (ctypes.c_int, [c_i32, c_ptr, c_size, c_ptr, c_size, c_i64, c_i64, c_ptr, c_i64,
                                                c_i32, c_ptr, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "mgp_expert_conditional_f16_batch": (ctypes.c_int, [c_i32, c_ptr, c_size, c_ptr, c_size, c_ptr, c_i64, c_ptr,
                                                        c_i64, c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size,
                                                        c_ptr, c_size, c_ptr, c_ptr]),
    "mgp_trsm_stats_f16x8": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_i64, c_i64, c_ptr, c_i64, c_i32,
                                            c_ptr, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64, c_ptr]),
    "mgp_expert_conditional_f16": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                  c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_expert_conditional_f16x8": (ctypes.c_int, [c_ptr, c_size, c_ptr, c_size, c_ptr, c_i64, c_ptr, c_i64,
                                                    c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_size, c_ptr]),
    "mgp_kl_workspace_bytes": (c_size, [c_i64, c_i32]),
    "mgp_qsqrt_workspace_bytes": (c_size, [c_i64, c_i32]),
    "mgp_qsqrt_images_kl_f16_batch": (ctypes.c_int, [c_i32, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr,
                                                     c_size, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_gauss_kl_white": (ctypes.c_int, [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32, c_ptr,
                                          c_ptr, c_size, c_ptr]),
    "mgp_elbo_workspace_bytes": (c_size, [c_i64]),
    "mgp_elbo_terms": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_i64, c_i32, c_i32, ctypes.c_float,
                                 ctypes.c_float, c_ptr, c_ptr, c_u64, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_elbo_terms_modified": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_i32, c_i32,
                                          ctypes.c_float, ctypes.c_float, c_ptr, c_ptr, c_u64, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_elbo_backward_workspace_bytes": (c_size, [c_i64, c_i32]),
    "mgp_elbo_terms_backward": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_i64, c_i32, c_i32,
                                          ctypes.c_float, ctypes.c_float, c_ptr, c_ptr, c_u64, c_i64, ctypes.c_float, c_ptr, c_i64,
                                          c_ptr, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_elbo_combine": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, ctypes.c_double, ctypes.c_double, c_ptr,
                                        c_ptr, c_ptr]),
    "mgp_predict_epilogue": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_ptr,
                                            c_ptr, c_ptr, c_ptr]),
    "mgp_philox_noise": (ctypes.c_int, [c_u64, c_i64, c_i64, c_i32, c_i32, c_ptr, c_ptr, c_ptr]),
    "mgp_philox_normal2": (ctypes.c_int, [c_u64, c_i64, c_i64, c_i32, c_i32, c_ptr, c_ptr]),
    "mgp_predict_samples": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_i32, c_i32, ctypes.c_float,
                                      ctypes.c_float, c_ptr, c_ptr, c_ptr, c_u64, c_i64, c_ptr, c_ptr, c_ptr]),
    "mgp_elbo_terms_multiclass": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, ctypes.c_float, c_ptr, c_i64, c_i32, c_i32,
                                            ctypes.c_float, ctypes.c_float, c_ptr, c_ptr, c_u64, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_elbo_terms_multiclass_backward": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, ctypes.c_float, c_ptr, c_i64, c_i32, c_i32,
                                                     ctypes.c_float, ctypes.c_float, c_ptr, c_ptr, c_u64, c_i64, ctypes.c_float, c_ptr, c_i64,
                                                     c_ptr, c_ptr, c_size, c_ptr]),
    "mgp_multiclass_predict": (ctypes.c_int, [c_ptr, c_ptr, c_i64, c_i64, c_i32, ctypes.c_float, c_ptr, c_ptr,
                                              c_ptr]),
    "mgp_predict_samples_multiclass": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, ctypes.c_float, c_i64, c_i32, c_i32, ctypes.c_float,
                                                 ctypes.c_float, c_ptr, c_ptr, c_ptr, c_u64, c_i64, c_ptr, c_ptr, c_ptr]),
    "mgp_assign_logits": (ctypes.c_int, [c_ptr, c_ptr, c_i64, c_i64, c_i64, c_i32, c_i32, ctypes.c_float, c_ptr,
                                         c_u64, c_i64, c_ptr, c_ptr]),
    "mgp_relaxed_onehot_sample": (ctypes.c_int, [c_ptr, c_i64, c_i32, c_i32, ctypes.c_float, c_ptr, c_u64, c_i64,
                                                 c_ptr, c_ptr]),
    "mgp_e_log_p_y": (ctypes.c_int, [c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, ctypes.c_float,
                                     c_ptr, c_i64, c_i32, c_i32, c_ptr, c_ptr]),
}

_lib = None


def header_symbols(path=HEADER_PATH):
    """Every function name declared in include/mgp_hip.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mgp_[a-z0-9_]+)\s*\(", text)))


def load():
    """Load libmgp_hip.so once (no HIP call is made by loading)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MGPLibraryError(
            f"{LIB_PATH} not found: build it with `python -m modulatedgps_amd.build` "
            "(there is no CPU fallback)")
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    except OSError as e:
        raise MGPLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(name, status):
    if status != 0:
        msg = load().mgp_status_string(status).decode()
        raise MGPError(name, status, msg)


def call(name, *args):
    """Call an int-returning entry point and raise MGPError on failure."""
    fn = getattr(load(), name)
    check(name, fn(*args))
