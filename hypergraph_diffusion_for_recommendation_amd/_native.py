"""ctypes binding of libhgd.so (the C ABI declared in include/hgd.h).

The product path goes through this module only: there is no CPU or PyTorch fallback. If the
shared library is missing the first call raises ``HGDNativeError`` telling how to build it
(``python -c "import __graft_entry__ as g; g.build()"`` or ``make -C .../csrc``).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HGD_LIB_PATH", os.path.join(_HERE, "_lib", "libhgd.so"))

c_void_p = ctypes.c_void_p
c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_f32 = ctypes.c_float
c_f64 = ctypes.c_double
c_size = ctypes.c_size_t

HGD_OK = 0
EPI_NONE, EPI_LEAKY_RELU, EPI_RELU = 0, 1, 2
_STATUS_NAMES = {0: "HGD_OK", 1: "HGD_ERR_INVALID_ARG", 2: "HGD_ERR_HIP",
                 3: "HGD_ERR_UNSUPPORTED", 4: "HGD_ERR_WORKSPACE"}


class HGDNativeError(RuntimeError):
    """Raised when libhgd is missing or a call returns a non-OK hgd_status."""


class SplitPlan(ctypes.Structure):
    """Mirror of ``hgd_split_plan`` (include/hgd.h)."""

    _fields_ = [
        ("threshold", c_i64),
        ("chunk", c_i32),
        ("flags", c_i32),
        ("n_heavy", c_i64),
        ("n_chunks", c_i64),
        ("heavy_rows", c_void_p),
        ("heavy_cptr", c_void_p),
        ("chunk_heavy", c_void_p),
    ]


class RowEpilogue(ctypes.Structure):
    """Mirror of ``hgd_row_epilogue`` (include/hgd.h)."""

    _fields_ = [
        ("act", c_i32),
        ("slope", c_f32),
        ("layer_norm", c_i32),
        ("ln_eps", c_f32),
        ("ln_gamma", c_void_p),
        ("ln_beta", c_void_p),
        ("out_scale", c_f32),
        ("res1", c_void_p),
        ("ld_res1", c_i64),
        ("res1_scale", c_f32),
        ("res2", c_void_p),
        ("ld_res2", c_i64),
        ("res2_scale", c_f32),
        ("act_out", c_void_p),
        ("ld_act", c_i64),
        ("stats", c_void_p),
        ("sum_res", c_void_p),
        ("ld_sum_res", c_i64),
        ("sum_out", c_void_p),
        ("ld_sum_out", c_i64),
    ]


class GemmRowsDesc(ctypes.Structure):
    """Mirror of ``hgd_gemm_rows_desc`` (include/hgd.h)."""

    _fields_ = [
        ("A", c_void_p),
        ("lda", c_i64),
        ("relu_mask", c_void_p),
        ("ldm", c_i64),
        ("B", c_void_p),
        ("bsk", c_i64),
        ("bsn", c_i64),
        ("bias", c_void_p),
        ("relu", c_i32),
        ("accumulate", c_i32),
        ("Y", c_void_p),
        ("ldy", c_i64),
        ("rows", c_i64),
        ("K", c_i32),
        ("N", c_i32),
        ("drop_seed", c_void_p),
        ("drop_keep", c_f32),
        ("drop_scale", c_f32),
        ("res", c_void_p),
        ("ldres", c_i64),
        ("Y2", c_void_p),
        ("ldy2", c_i64),
        ("row_inv", c_void_p),
        ("binarize_a", c_i32),
        ("b_row_count", c_void_p),
        ("b_scale", ctypes.c_float),
        ("a_drop_seed", c_void_p),
        ("a_drop_keep", c_f32),
        ("a_drop_scale", c_f32),
    ]


class GemmTnDesc(ctypes.Structure):
    """Mirror of ``hgd_gemm_tn_desc`` (include/hgd.h)."""

    _fields_ = [
        ("A", c_void_p),
        ("lda", c_i64),
        ("relu_mask", c_void_p),
        ("ldm", c_i64),
        ("B", c_void_p),
        ("ldb", c_i64),
        ("rows", c_i64),
        ("M", c_i32),
        ("N", c_i32),
        ("C", c_void_p),
        ("colsum_A", c_void_p),
        ("binarize_a", c_i32),
        ("b_row_scale", c_void_p),
        ("c_scale", ctypes.c_float),
        ("b_drop_seed", c_void_p),
        ("b_drop_keep", c_f32),
        ("b_drop_scale", c_f32),
    ]


class UniqueJob(ctypes.Structure):
    """Mirror of ``hgd_unique_job`` (include/hgd.h)."""

    _fields_ = [
        ("x_f32", c_void_p),
        ("x_i64", c_void_p),
        ("n", c_i64),
        ("capacity", c_i64),
        ("out", c_void_p),
        ("n_out", c_void_p),
        ("workspace", c_void_p),
        ("workspace_bytes", c_size),
    ]


class InfonceTerm(ctypes.Structure):
    """Mirror of ``hgd_infonce_term`` (include/hgd.h)."""

    _fields_ = [
        ("E1", c_void_p),
        ("ld1", c_i64),
        ("E2", c_void_p),
        ("ld2", c_i64),
        ("n_rows", c_i64),
        ("nodes", c_void_p),
        ("capacity", c_i64),
        ("batch_count", c_void_p),
        ("P1", c_void_p),
        ("P2", c_void_p),
        ("inv_norm1", c_void_p),
        ("inv_norm2", c_void_p),
        ("pos_logit", c_void_p),
        ("deno", c_void_p),
        ("loss", c_void_p),
        ("dX1", c_void_p),
        ("dX2", c_void_p),
        ("dE1", c_void_p),
        ("ldE1", c_i64),
        ("dE2", c_void_p),
        ("ldE2", c_i64),
        ("workspace", c_void_p),
        ("workspace_bytes", c_size),
    ]


class AdamTensor(ctypes.Structure):
    """Mirror of ``hgd_adam_tensor`` (include/hgd.h)."""

    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p),
                ("exp_avg_sq", c_void_p), ("n", c_i64)]


class MaskedSum(ctypes.Structure):
    """Mirror of ``hgd_masked_sum`` (include/hgd.h)."""

    _fields_ = [("dy", c_void_p * 8), ("mask", c_void_p * 8), ("out", c_void_p), ("n", c_i64),
                ("count", c_i32), ("scale", c_f32)]


class IncidenceView(ctypes.Structure):
    """Mirror of ``hgd_incidence_view`` (include/hgd.h)."""

    _fields_ = [
        ("n_rows", c_i64),
        ("n_cols", c_i64),
        ("nnz", c_i64),
        ("rowptr", c_void_p),
        ("col", c_void_p),
        ("val", c_void_p),
        ("colptr", c_void_p),
        ("row_t", c_void_p),
        ("val_t", c_void_p),
        ("perm_t", c_void_p),
    ]


SCALE_NONE, SCALE_MEAN, SCALE_SYM, SCALE_WMEAN, SCALE_WSYM = 0, 1, 2, 3, 4
SCALE_KINDS = {None: SCALE_NONE, "mean": SCALE_MEAN, "sym": SCALE_SYM, "wmean": SCALE_WMEAN,
               "wsym": SCALE_WSYM}
SIDE_ROWS, SIDE_COLS = 0, 1
COMM_ID_BYTES = 128
P2P_HANDLE_BYTES = 4096
_PP = ctypes.POINTER(c_void_p)

# name -> (restype, argtypes); every symbol of include/hgd.h appears here.
_SIGNATURES = {
    "hgd_version": (c_i32, []),
    "hgd_set_tuning": (c_i32, [c_i32, c_i32]),
    "hgd_get_last_error_string": (ctypes.c_char_p, []),
    "hgd_split_plan_count": (c_i32, [c_void_p, c_i64, c_i64, c_i32, c_void_p, c_void_p]),
    "hgd_split_plan_workspace_size": (c_size, [c_i64]),
    "hgd_split_plan_build": (c_i32, [c_void_p, c_i64, c_i64, c_i32, c_void_p, c_void_p, c_void_p,
                                     c_i64, c_i64, c_void_p, c_size, c_void_p]),
    "hgd_spmm_workspace_size": (c_size, [ctypes.POINTER(SplitPlan), c_i32]),
    "hgd_spmm": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_i64, c_i64,
                         c_void_p, c_i64, c_void_p, c_i64, c_i32, c_i32, c_f32,
                         ctypes.POINTER(SplitPlan), c_void_p, c_size, c_void_p]),
    "hgd_spmm_blocks_for": (c_i32, [c_i64, c_i32]),
    "hgd_spmm_col_blocks_workspace_size": (c_size, [c_i64, c_i32]),
    "hgd_spmm_col_blocks": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_i32, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_spmm_blocked": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_i64,
                                 c_i64, c_void_p, c_i64, c_void_p, c_i64, c_i32, c_i32, c_f32,
                                 c_i32, c_void_p]),
    "hgd_spmm_masked": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_f32, c_void_p, c_i64,
                                c_i64, c_i64, c_i64, c_void_p, c_i64, c_void_p, c_i64, c_i32,
                                c_i32, c_f32, ctypes.POINTER(SplitPlan), c_void_p, c_size,
                                c_void_p]),
    "hgd_spmm_masked_fused": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_f32, c_void_p,
                                      c_i64, c_i64, c_i64, c_i64, c_void_p, c_i64, c_void_p,
                                      c_i64, c_i32, ctypes.POINTER(RowEpilogue),
                                      ctypes.POINTER(SplitPlan), c_void_p, c_size, c_void_p]),
    "hgd_spmm_fused": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_i64,
                               c_i64, c_void_p, c_i64, c_void_p, c_i64, c_i32,
                               ctypes.POINTER(RowEpilogue), ctypes.POINTER(SplitPlan), c_void_p,
                               c_size, c_void_p]),
    "hgd_row_epilogue_forward": (c_i32, [c_void_p, c_i64, c_i64, c_i32,
                                         ctypes.POINTER(RowEpilogue), c_void_p, c_i64,
                                         c_void_p]),
    "hgd_row_epilogue_backward_workspace_size": (c_size, [c_i64, c_i32]),
    "hgd_row_epilogue_backward": (c_i32, [c_void_p, c_i64, c_void_p, c_i64, c_void_p, c_void_p,
                                          c_i64, c_i32, c_i32, c_f32, c_i32, c_f32, c_void_p,
                                          c_i64, c_void_p, c_void_p, c_void_p, c_size,
                                          c_void_p]),
    "hgd_linear_forward": (c_i32, [c_void_p, c_i64, c_i64, c_i32, c_void_p, c_i64, c_i32,
                                   c_void_p, c_i32, c_void_p, c_i64, c_void_p]),
    "hgd_linear_backward_data": (c_i32, [c_void_p, c_i64, c_void_p, c_i64, c_i64, c_i32,
                                         c_void_p, c_i64, c_i32, c_void_p, c_i64, c_void_p]),
    "hgd_linear_backward_weight_workspace_size": (c_size, [c_i64, c_i32, c_i32]),
    "hgd_linear_backward_weight": (c_i32, [c_void_p, c_i64, c_void_p, c_i64, c_void_p, c_i64,
                                           c_i64, c_i32, c_i32, c_void_p, c_void_p, c_void_p,
                                           c_size, c_void_p]),
    "hgd_gemm_rows": (c_i32, [ctypes.POINTER(GemmRowsDesc), c_i32, c_void_p]),
    "hgd_gemm_tn_workspace_size": (c_size, [ctypes.POINTER(GemmTnDesc), c_i32]),
    "hgd_gemm_tn": (c_i32, [ctypes.POINTER(GemmTnDesc), c_i32, c_void_p, c_size, c_void_p]),
    "hgd_infonce_workspace_size": (c_size, [c_i64, c_i32]),
    "hgd_infonce_forward": (c_i32, [c_void_p, c_i64, c_void_p, c_i64, c_i64, c_void_p, c_i64,
                                    c_i32, c_f32, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_infonce_backward": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64,
                                     c_i32, c_f32, c_void_p, c_void_p, c_void_p, c_void_p,
                                     c_size, c_void_p]),
    "hgd_infonce_forward_n": (c_i32, [c_void_p, c_i64, c_void_p, c_i64, c_i64, c_void_p, c_i64,
                                      c_void_p, c_i32, c_f32, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size,
                                      c_void_p]),
    "hgd_infonce_backward_n": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i64,
                                       c_void_p, c_i32, c_f32, c_void_p, c_void_p, c_i64,
                                       c_void_p, c_i64, c_void_p, c_i64, c_void_p, c_size,
                                       c_void_p]),
    "hgd_infonce_forward_group": (c_i32, [ctypes.POINTER(InfonceTerm), c_i32, c_i32, c_f32,
                                          c_void_p]),
    "hgd_infonce_backward_group": (c_i32, [ctypes.POINTER(InfonceTerm), c_i32, c_i32, c_f32,
                                           c_void_p, c_void_p]),
    "hgd_bernoulli_mask_dev_pair": (c_i32, [c_void_p, c_void_p, c_i64, c_f32, c_void_p, c_void_p,
                                            c_void_p]),
    "hgd_bernoulli_mask_dev": (c_i32, [c_void_p, c_i64, c_f32, c_void_p, c_void_p]),
    "hgd_dropedge_fill_tail": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p]),
    "hgd_ingest_read": (c_i32, [ctypes.c_char_p, c_i32, c_i32, ctypes.POINTER(c_void_p)]),
    "hgd_ingest_count": (c_i64, [c_void_p]),
    "hgd_ingest_copy": (c_i32, [c_void_p, c_void_p, c_void_p]),
    "hgd_ingest_free": (None, [c_void_p]),
    "hgd_remap_workspace_size": (c_size, [c_i64]),
    "hgd_remap_first_appearance": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_size, c_void_p]),
    "hgd_coo_coalesce_workspace_size": (c_size, [c_i64]),
    "hgd_coo_coalesce": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_i64, c_void_p, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_normalize_values": (c_i32, [c_void_p, c_void_p, c_void_p, c_i64, c_void_p, c_void_p,
                                     c_void_p, c_void_p]),
    "hgd_index_narrow": (c_i32, [c_void_p, c_i64, c_i64, c_void_p, c_void_p, c_void_p]),
    "hgd_sort_perm_workspace_size": (c_size, [c_i64]),
    "hgd_sort_perm": (c_i32, [c_void_p, c_i64, c_i64, c_void_p, c_void_p, c_void_p, c_size,
                              c_void_p]),
    "hgd_rowptr_from_sorted": (c_i32, [c_void_p, c_i64, c_i64, c_void_p, c_void_p]),
    "hgd_check_sorted": (c_i32, [c_void_p, c_i64, c_i64, c_void_p, c_void_p]),
    "hgd_expand_rows": (c_i32, [c_void_p, c_i64, c_i64, c_void_p, c_void_p]),
    "hgd_gather_u8": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_void_p]),
    "hgd_gather32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p, c_void_p]),
    "hgd_degree_scale": (c_i32, [c_void_p, c_void_p, c_i64, c_f64, c_void_p, c_void_p]),
    "hgd_edge_values": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_void_p,
                                c_void_p]),
    "hgd_dropedge_workspace_size": (c_size, [c_i64]),
    "hgd_dropedge_compact": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i64, c_f32,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size,
                                     c_void_p]),
    "hgd_bernoulli_mask": (c_i32, [ctypes.c_uint64, c_i64, c_f32, c_void_p, c_void_p]),
    "hgd_dropedge_structure_workspace_size": (c_size, [c_i64]),
    "hgd_dropedge_structure": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_i64, c_i64, c_i64, c_void_p, c_f32,
                                       c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_dense_threshold_workspace_size": (c_size, [c_i64]),
    "hgd_dense_threshold_rowptr": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_f32, c_i32,
                                           c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_dense_threshold_fill": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_f32, c_i32, c_void_p,
                                         c_void_p, c_void_p, c_void_p]),
    "hgd_mask_scores": (c_i32, [c_void_p, c_i64, c_i64, c_void_p, c_void_p, c_void_p, c_f32,
                                c_void_p]),
    "hgd_topk_rows": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_i32, c_void_p, c_void_p,
                              c_void_p]),
    "hgd_rank_metrics": (c_i32, [c_void_p, c_i64, c_i64, c_i32, c_void_p, c_void_p,
                                 ctypes.POINTER(c_i32), c_i32, c_void_p, c_void_p, c_void_p,
                                 c_void_p]),
    "hgd_py_shuffle": (c_i32, [c_void_p, c_void_p, c_i64]),
    "hgd_sample_pairwise": (c_i32, [c_void_p, c_void_p, c_i64, c_i64, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_i64, c_i64, c_i32, c_void_p, c_void_p,
                                    c_void_p]),
    "hgd_torch_cpu_state_bytes": (c_size, []),
    "hgd_torch_cpu_jump_selfcheck": (c_i32, [c_i64]),
    "hgd_torch_cpu_keep_mask": (c_i32, [c_void_p, c_i64, c_i64, c_f32, c_void_p,
                                        ctypes.POINTER(c_i64)]),
    "hgd_torch_cpu_keep_mask_threads": (c_i32, [c_void_p, c_i64, c_i64, c_f32, c_void_p,
                                                ctypes.POINTER(c_i64), c_i32]),
    "hgd_epilogue_apply":(c_i32, [c_void_p, c_i64, c_i32, c_f32, c_void_p, c_void_p]),
    "hgd_epilogue_backward": (c_i32, [c_void_p, c_void_p, c_i64, c_i32, c_f32, c_void_p,
                                      c_void_p]),
    "hgd_sum_slices": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_void_p, c_void_p]),
    "hgd_sum_arrays": (c_i32, [c_void_p, c_i32, c_i64, c_void_p, c_void_p]),
    "hgd_adam_step": (c_i32, [c_void_p, c_i32, c_void_p, c_void_p, c_i32, c_void_p]),
    "hgd_dropout_apply": (c_i32, [c_void_p, c_i64, c_void_p, c_f32, c_f32, c_void_p, c_void_p]),
    "hgd_masked_scale_sum": (c_i32, [c_void_p, c_i32, c_void_p]),
    "hgd_bpr_workspace_size": (c_size, [c_i64, c_i64]),
    "hgd_bpr_forward": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_i32, c_void_p, c_void_p,
                                c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_bpr_backward": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_i32, c_void_p, c_void_p,
                                 c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_i64, c_void_p,
                                 c_size, c_void_p]),
    "hgd_unique_workspace_size": (c_size, [c_i64]),
    "hgd_unique_i64": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_size, c_void_p]),
    "hgd_unique_trunc_f32": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_size,
                                     c_void_p]),
    "hgd_unique_dev_i64": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_size,
                                   c_void_p]),
    "hgd_unique_dev_trunc_f32": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_size,
                                         c_void_p]),
    "hgd_unique_dev_group": (c_i32, [c_void_p, c_i32, c_void_p]),
    "hgd_unique_sort_i64": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_size,
                                    c_void_p]),
    "hgd_unique_sort_trunc_f32": (c_i32, [c_void_p, c_i64, c_void_p, c_void_p, c_void_p, c_size,
                                          c_void_p]),
    # incidence objects, conv2hop, RCCL exchange
    "hgd_incidence_create": (c_i32, [c_void_p, c_void_p, c_void_p, c_i64, c_i64, c_i64, _PP,
                                     c_void_p]),
    "hgd_incidence_from_dense": (c_i32, [c_void_p, c_i64, c_i64, c_i64, c_f32, c_i32, c_i32,
                                         _PP, c_void_p]),
    "hgd_incidence_dropedge": (c_i32, [c_void_p, c_void_p, c_f32, _PP, c_void_p]),
    "hgd_incidence_destroy": (None, [c_void_p]),
    "hgd_incidence_get_view": (c_i32, [c_void_p, ctypes.POINTER(IncidenceView)]),
    "hgd_incidence_scale": (c_i32, [c_void_p, c_i32, c_i32, _PP]),
    "hgd_incidence_prepare": (c_i32, [c_void_p, ctypes.c_uint32, c_void_p]),
    "hgd_incidence_workspace_size": (c_size, [c_void_p, c_i32]),
    "hgd_incidence_spmm": (c_i32, [c_void_p, c_i32, c_void_p, c_i64, c_void_p, c_i64, c_i32,
                                   c_void_p, c_i32, c_f32, c_void_p, c_size, c_void_p]),
    "hgd_comm_get_unique_id": (c_i32, [c_void_p]),
    "hgd_comm_create": (c_i32, [c_void_p, c_i32, c_i32, _PP]),
    "hgd_comm_destroy": (None, [c_void_p]),
    "hgd_comm_set_chunks": (c_i32, [c_void_p, c_i32]),
    "hgd_exchange_allreduce": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p]),
    "hgd_p2p_create": (c_i32, [c_i32, c_i32, c_i64, c_i32, _PP]),
    "hgd_p2p_destroy": (None, [c_void_p]),
    "hgd_p2p_export": (c_i32, [c_void_p, c_void_p]),
    "hgd_p2p_open": (c_i32, [c_void_p, c_void_p]),
    "hgd_p2p_slot": (c_void_p, [c_void_p, c_i32]),
    "hgd_p2p_set_timeout": (c_i32, [c_void_p, ctypes.c_double]),
    "hgd_p2p_allreduce": (c_i32, [c_void_p, c_i32, c_i64, c_void_p, c_void_p]),
    "hgd_p2p_check": (c_i32, [c_void_p]),
    "hgd_p2p_price_local": (c_i32, [c_i32, c_i64, c_i32, c_i32, ctypes.POINTER(c_f32),
                                    ctypes.POINTER(c_f32), c_void_p]),
    "hgd_comm_create_p2p": (c_i32, [c_void_p, c_i32, c_i32, _PP]),
    "hgd_comm_set_slice_width": (c_i32, [c_void_p, c_i32]),
    "hgd_p2p_poll": (c_i32, [c_void_p]),
    "hgd_p2p_n_slots": (c_i32, [c_void_p]),
    "hgd_p2p_max_count": (c_i64, [c_void_p]),
    "hgd_p2p_block_range": (c_i32, [c_i64, c_i32, c_i32, ctypes.POINTER(c_i64),
                                    ctypes.POINTER(c_i64)]),
    "hgd_p2p_gather_index": (c_i32, [c_i64, c_i32, c_i32, c_i64, ctypes.POINTER(c_i64),
                                     ctypes.POINTER(c_i32)]),
    "hgd_incidence_globalize_columns": (c_i32, [c_void_p, c_void_p, c_void_p]),
    "hgd_conv2hop_workspace_size": (c_size, [c_void_p, c_i32, c_i32]),
    "hgd_conv2hop_forward": (c_i32, [c_void_p, c_i32, c_i32, c_i32, c_void_p, c_i64, c_i32,
                                     c_void_p, c_i64, c_i32, c_f32, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_size, c_void_p]),
    "hgd_conv2hop_backward": (c_i32, [c_void_p, c_i32, c_i32, c_i32, c_void_p, c_i64, c_i32,
                                      c_void_p, c_i32, c_f32, c_void_p, c_i64, c_void_p,
                                      c_void_p, c_size, c_void_p]),
}

_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Loads libhgd.so once and binds every ABI symbol; raises HGDNativeError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HGDNativeError(
                f"libhgd.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        # optional process-wide tuning overrides (hgd_set_tuning keys 1 .. 18)
        for key, env in ((1, "HGD_SPMM_UNROLL"), (2, "HGD_SPMM_POLICY"),
                         (3, "HGD_SPMM_PASS_COLS"), (4, "HGD_ROWGEMM_BLOCKS"),
                         (5, "HGD_SPLITK_ROWS"), (6, "HGD_GEMM_EXACT"),
                         (7, "HGD_X3_COLS"), (8, "HGD_X3_SPLITK"), (9, "HGD_X3S_TILES"),
                         (10, "HGD_P2P_SEGMENT_MB"), (11, "HGD_P2P_CACHED"),
                         (12, "HGD_CPU_RNG_THREADS"), (13, "HGD_X3P_QUEUE"),
                         (14, "HGD_P2P_GRID"), (15, "HGD_MASK_PAIR"), (16, "HGD_MASK_DIV"),
                         (17, "HGD_SPMM_PASS_INTERLEAVE"), (18, "HGD_SPMM_BLOCKED_SEG")):
            if os.environ.get(env):
                st = lib.hgd_set_tuning(key, int(os.environ[env]))
                if st != HGD_OK:
                    raise HGDNativeError(f"{env}={os.environ[env]}: "
                                         f"{lib.hgd_get_last_error_string().decode()}")
        _lib = lib
    return _lib


def symbols():
    return list(_SIGNATURES)


def check(status: int, what: str) -> None:
    if status != HGD_OK:
        msg = load().hgd_get_last_error_string().decode(errors="replace")
        raise HGDNativeError(f"{what}: {_STATUS_NAMES.get(status, status)}: {msg}")


def ptr(t) -> int | None:
    """Device pointer of a tensor (None for None)."""
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    """The raw ``hipStream_t`` of torch's current stream on ``device`` (a torch.device, an index
    or None for the current device). torch's ``current_stream(device).cuda_stream`` builds a
    Stream object per call (≈ 10 µs — a quarter of an eager hop's host time at dataset sizes);
    the raw getter returns the same handle in well under a microsecond."""
    import torch
    if _RAW_STREAM is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return _RAW_STREAM(idx)
    return torch.cuda.current_stream(device).cuda_stream


def _raw_stream_getter():
    try:
        import torch
        return getattr(torch._C, "_cuda_getCurrentRawStream", None)
    except Exception:  # pragma: no cover - torch without the HIP module
        return None


_RAW_STREAM = _raw_stream_getter()


# ---------------------------------------------------------------------------------------------
# Views of library-owned device memory as torch tensors (DLPack, no copy): the send slots of an
# hgd_p2p exchange are written directly by the hop kernels through such views.
# ---------------------------------------------------------------------------------------------
class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(c_i64)),
                ("strides", ctypes.POINTER(c_i64)), ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    _fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", c_void_p), ("deleter", c_void_p)]


_DL_CPU, _DL_ROCM = 1, 10
_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [c_void_p, ctypes.c_char_p, c_void_p]


def float_view(address: int, shape, device, on_release=None) -> "torch.Tensor":
    """A contiguous float32 tensor over ``address`` (device memory the library owns, or host
    memory for ``device`` = cpu) without copying. ``on_release()`` runs when torch releases the
    tensor's STORAGE — after the last tensor or view sharing it is gone, which may be well after
    the returned tensor object — through the DLPack record's deleter: the owner of the memory
    counts its live views this way and frees the memory only once none is left (a view can never
    reach freed memory). Nothing here references the owner, so a view does not keep its owner's
    Python object alive (no reference cycle through a global)."""
    import torch
    device = torch.device(device)
    shape = tuple(int(s) for s in shape)
    rec = _DLManagedTensor()
    shp = (c_i64 * len(shape))(*shape)
    rec.dl_tensor.data = address
    if device.type == "cpu":
        rec.dl_tensor.device = _DLDevice(_DL_CPU, 0)
    else:
        rec.dl_tensor.device = _DLDevice(_DL_ROCM, device.index if device.index is not None
                                         else torch.cuda.current_device())
    rec.dl_tensor.ndim = len(shape)
    rec.dl_tensor.dtype = _DLDataType(2, 32, 1)  # kDLFloat, 32 bits
    rec.dl_tensor.shape = ctypes.cast(shp, ctypes.POINTER(c_i64))
    rec.dl_tensor.strides = None  # compact row-major
    rec.dl_tensor.byte_offset = 0
    rec.manager_ctx = None
    rec.deleter = ctypes.cast(_DL_DELETER, c_void_p)
    # the record and its shape array live until torch calls the deleter with the record
    _LIVE_RECORDS[ctypes.addressof(rec)] = (rec, shp, on_release)
    cap = _PyCapsule_New(ctypes.addressof(rec), b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(cap)


_LIVE_RECORDS = {}


@ctypes.CFUNCTYPE(None, c_void_p)
def _DL_DELETER(address, _live=_LIVE_RECORDS):
    """DLManagedTensor.deleter: torch released the storage of a float_view."""
    try:
        entry = _live.pop(address, None)
        if entry is not None and entry[2] is not None:
            entry[2]()
    except Exception:  # noqa: BLE001 — never raise into torch's storage release
        pass


# torch may release a view's storage during interpreter teardown, after this module's globals
# are gone: one extra reference keeps the thunk (and, through its default, the record table)
# alive for the life of the process, so the deleter is never a freed callback. The callbacks it
# runs only do bookkeeping (sharded._P2PHandle.view_gone): no HIP call inside torch's release.
ctypes.pythonapi.Py_IncRef(ctypes.py_object(_DL_DELETER))


def live_views() -> int:
    """float_view storages torch has not released yet (tests)."""
    return len(_LIVE_RECORDS)
