"""ctypes binding of ``libgnnmp.so`` — the C ABI declared in ``include/gnnmp.h``.

The library is built in-tree (``make -C elliptic_gnn_project_amd/csrc``) and loaded
from the package directory.  There is no fallback: if the shared object is missing
or fails to load, every op raises.  ``torch`` is imported first so that the HIP
runtime torch ships (soname ``libamdhip64.so.7``) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (loads the HIP runtime before libgnnmp)

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["GNNMP_LIB"]) if os.environ.get("GNNMP_LIB") else PKG_DIR / "libgnnmp.so"  # (GNNMP_LIB: A/B builds)
ABI_VERSION = 26

# gnn_dtype
DTYPE_F32 = 0
DTYPE_BF16 = 1

# gnn_gemm_math
MATH_SPLIT_BF16 = 0
MATH_F32 = 1
MATH_HALF_PAIR = 2  # ABI 23: f32 operands split into half-pair f16 in the kernel (3 products)

# gnn_planes_format
PLANES_SPLIT_BF16 = 0
PLANES_HALF_PAIR = 1

# gnn_status
GNN_OK = 0
_STATUS_EXC = {
    1: ValueError,
    2: IndexError,
    3: RuntimeError,
    4: RuntimeError,
    5: NotImplementedError,
}

# gnn_loop_mode
LOOPS_KEEP = 0
LOOPS_REPLACE = 1

# gnn_agg_mode
AGG_SUM = 0
AGG_MEAN = 1
AGG_MEAN_BWD = 2
AGG_GCN = 3
AGG_EDGE_W = 4

c_i64 = ctypes.c_int64
c_i32 = ctypes.c_int32
c_ptr = ctypes.c_void_p
c_size = ctypes.c_size_t


class GnnSplit(ctypes.Structure):
    _fields_ = [
        ("seg_len", c_i32),
        ("reserved", c_i32),
        ("num_long", c_i64),
        ("num_pieces", c_i64),
        ("ptr", c_ptr),
        ("nbr", c_ptr),
        ("piece0", c_ptr),
        ("piece_seg", c_ptr),
        ("long_seg", c_ptr),
        ("order", c_ptr),
    ]


class GnnGraph(ctypes.Structure):
    _fields_ = [
        ("num_nodes", c_i64),
        ("num_slots", c_i64),
        ("rowptr", c_ptr),
        ("col", c_ptr),
        ("colptr", c_ptr),
        ("row", c_ptr),
        ("csc2csr", c_ptr),
        ("csr_split", ctypes.POINTER(GnnSplit)),
        ("csc_split", ctypes.POINTER(GnnSplit)),
    ]


class GnnAggParams(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int),
        ("transpose", c_i32),
        ("nodew", c_ptr),
        ("ew", c_ptr),
        ("heads", c_i32),
        ("addend", c_ptr),
        ("ld_add", c_i64),
        ("bias", c_ptr),
        ("relu", c_i32),
        ("part", c_ptr),
        ("part_bytes", c_size),
        ("dropout_p", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("seed_ptr", c_ptr),
        ("addend2", c_ptr),
        ("ld_add2", c_i64),
    ]


class GnnGemmNTParams(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64),
        ("a1", c_ptr), ("lda1", c_i64), ("k1", c_i64),
        ("a2", c_ptr), ("lda2", c_i64), ("k2", c_i64),
        ("bt", c_ptr), ("ldb", c_i64),
        ("w1", c_ptr), ("w2", c_ptr), ("ldw1", c_i64), ("ldw2", c_i64),
        ("c", c_ptr), ("ldc", c_i64),
        ("bias", c_ptr),
        ("relu", c_i32),
        ("dropout_p", ctypes.c_float),
        ("seed", ctypes.c_uint64),
        ("seed_ptr", c_ptr),
        ("proj", c_ptr), ("nproj", c_i32), ("z", c_ptr), ("ldz", c_i64),
        ("math", c_i32),
        ("workspace", c_ptr), ("workspace_bytes", c_size),
        ("a_dtype", c_i32), ("c_dtype", c_i32),
        ("mask", c_ptr), ("ldmask", c_i64), ("mask_scale", ctypes.c_float),
        ("a_planes", c_ptr), ("planes_ld", c_i64), ("planes_stride", c_i64), ("planes_col2", c_i64),
        ("planes_format", c_i32), ("keep_mask", c_ptr), ("b_ready", c_i32), ("planes_exp", c_i32),
        ("colsum_part", c_ptr), ("colsum_cap", c_i64),
        ("row_exp", c_ptr),
    ]


class GnnGemmTNParams(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("Nr", c_i64),
        ("g", c_ptr), ("ldg", c_i64),
        ("dz", c_ptr), ("lddz", c_i64),
        ("proj", c_ptr), ("nproj", c_i32),
        ("h", c_ptr), ("ldh", c_i64), ("hscale", ctypes.c_float),
        ("gout", c_ptr), ("ldgout", c_i64),
        ("a1", c_ptr), ("lda1", c_i64), ("k1", c_i64),
        ("a2", c_ptr), ("lda2", c_i64), ("k2", c_i64),
        ("math", c_i32),
        ("a_dtype", c_i32), ("h_dtype", c_i32),
        ("a_planes", c_ptr), ("planes_ld", c_i64), ("planes_stride", c_i64), ("planes_col2", c_i64),
        ("planes_format", c_i32), ("g_dtype", c_i32), ("planes_exp", c_i32),
        ("sq_partial", c_ptr), ("sq_step", c_ptr), ("sq_skip_lo", c_i64), ("sq_skip_hi", c_i64), ("sq_cap", c_i64),
        ("row_exp", c_ptr),
        ("g_rowmax", c_ptr),  # ABI 25
        ("dz_graph", c_ptr), ("dz_u", c_ptr), ("ldu", c_i64), ("dz_cols", c_i32),  # ABI 26
    ]


ROWMAX_ROWS = 16  # GNN_ROWMAX_ROWS (ABI 25)


# gnn_act
ACT_NONE = 0
ACT_ELU = 1


class GnnGatFwdParams(ctypes.Structure):
    _fields_ = [
        ("heads", c_i32), ("chans", c_i32), ("concat", c_i32),
        ("slope", ctypes.c_float),
        ("xh", c_ptr), ("ld_xh", c_i64),
        ("att_src", c_ptr), ("att_dst", c_ptr),
        ("bias", c_ptr),
        ("act", ctypes.c_int),
        ("dropout_p", ctypes.c_float),
        ("seed", ctypes.c_uint64), ("seed_ptr", c_ptr),
        ("a_src", c_ptr), ("a_dst", c_ptr),
        ("alpha", c_ptr),
        ("out", c_ptr), ("ldo", c_i64),
        ("edge_w", c_ptr),
        ("proj", c_ptr), ("nproj", c_i32), ("z", c_ptr), ("ldz", c_i64),
    ]


ADAM_MAX_TENSORS = 24


class GnnAdamTensor(ctypes.Structure):
    _fields_ = [("param", c_ptr), ("grad", c_ptr), ("exp_avg", c_ptr), ("exp_avg_sq", c_ptr), ("numel", c_i64)]


class GnnAdamGroup(ctypes.Structure):
    _fields_ = [
        ("num_tensors", c_i32),
        ("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double), ("eps", ctypes.c_double),
        ("weight_decay", ctypes.c_double), ("max_norm", ctypes.c_double),
        ("tensors", GnnAdamTensor * ADAM_MAX_TENSORS),
        ("skip_nonfinite", c_i32),
        ("bump_counter", c_ptr),
        ("loss_partial", c_ptr), ("loss_nblk", c_i32), ("loss_scale", ctypes.c_float), ("loss_out", c_ptr),
        ("grad_sq_partial", c_ptr), ("grad_sq_nblk", c_i32),
    ]


# name -> (restype, argtypes).  Mirrors include/gnnmp.h one to one; the CPU test
# suite checks that every function declared in the header appears here and is exported.
SIGNATURES = {
    "gnn_abi_version": (ctypes.c_int, []),
    "gnn_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "gnn_last_error": (ctypes.c_char_p, []),
    "gnn_graph_workspace_size": (ctypes.c_int, [c_i64, c_i64, ctypes.POINTER(c_size)]),
    "gnn_graph_build": (
        ctypes.c_int,
        [c_ptr, c_i64, c_i64, ctypes.c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_split_workspace_size": (ctypes.c_int, [c_i64, ctypes.POINTER(c_size)]),
    "gnn_split_count": (ctypes.c_int, [c_ptr, c_i64, c_i32, c_ptr, c_ptr]),
    "gnn_split_build": (
        ctypes.c_int,
        [c_ptr, c_ptr, c_i64, c_i32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_in_degree_f32": (ctypes.c_int, [ctypes.POINTER(GnnGraph), c_ptr, c_ptr]),
    "gnn_gcn_norm_f32": (ctypes.c_int, [ctypes.POINTER(GnnGraph), c_ptr, c_ptr]),
    "gnn_aggregate_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), ctypes.POINTER(GnnAggParams), c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    ),
    "gnn_aggregate_bf16": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), ctypes.POINTER(GnnAggParams), c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    ),
    "gnn_sage_mean_fwd_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    ),
    "gnn_split_planes_f32": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i64, c_ptr]),
    "gnn_sage_mean_fwd_planes": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr],
    ),
    "gnn_split_h2_f32": (ctypes.c_int, [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i64, c_i32, c_ptr]),
    "gnn_sage_mean_fwd_h2": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_i64, c_i64, c_i32,
         c_ptr, c_i64, ctypes.c_float, ctypes.c_uint64, c_ptr, ctypes.POINTER(GnnGemmNTParams),
         ctypes.POINTER(GnnSplit), c_ptr],
    ),
    "gnn_sage_out_mean_ce_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
         ctypes.c_float, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_sage_mean_bwd_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    ),
    "gnn_edge_dot_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_ptr],
    ),
    "gnn_gat_scores_f32": (
        ctypes.c_int,
        [c_i64, c_i32, c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    ),
    "gnn_gat_fwd_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_i32, c_i32, c_i32, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr,
         c_ptr, c_ptr, c_ptr, c_i64, c_ptr],
    ),
    "gnn_gat_fwd_fused_f32": (ctypes.c_int, [ctypes.POINTER(GnnGraph), ctypes.POINTER(GnnGatFwdParams), c_ptr]),
    "gnn_gat_out_ce_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), ctypes.POINTER(GnnGatFwdParams), c_ptr, c_ptr, c_ptr, ctypes.c_float, c_ptr, c_i64,
         c_ptr, c_ptr, c_ptr, c_size, c_ptr]),
    "gnn_gat_act_bwd_f32": (
        ctypes.c_int,
        [c_i64, c_i64, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr,
         c_i64, c_ptr],
    ),
    "gnn_gat_bwd_workspace_size": (ctypes.c_int, [c_i64, c_i64, c_i32, c_i32, ctypes.POINTER(c_size)]),
    "gnn_gat_bwd_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_i32, c_i32, c_i32, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
         c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_gat_bwd_act_proj_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_i32, c_i32, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
         c_i32, ctypes.c_float, ctypes.c_uint64, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i32, c_ptr, c_i64,
         c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_size, c_ptr]),
    "gnn_gat_bwd_act_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_i32, c_i32, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
         c_i32, ctypes.c_float, ctypes.c_uint64, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64,
         c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_gat_bwd_ew_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_i32, c_i32, c_i32, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
         c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_gemm_nt_workspace_size": (ctypes.c_int, [c_i64, c_i64, c_i64, ctypes.POINTER(c_size)]),
    "gnn_gemm_nt_f32": (ctypes.c_int, [ctypes.POINTER(GnnGemmNTParams), c_ptr]),
    "gnn_gemm_nt_prep_b": (ctypes.c_int, [ctypes.POINTER(GnnGemmNTParams), c_ptr]),
    "gnn_masked_ce_finish": (ctypes.c_int, [c_ptr, c_i32, ctypes.c_float, c_ptr, c_ptr]),
    "gnn_gemm_tn_workspace_size": (ctypes.c_int, [c_i64, c_i64, c_i64, c_i32, ctypes.POINTER(c_size)]),
    "gnn_gemm_tn_sq_blocks": (ctypes.c_int, [c_i64, ctypes.POINTER(c_i32)]),
    "gnn_gemm_tn_f32": (ctypes.c_int, [ctypes.POINTER(GnnGemmTNParams), c_ptr, c_ptr, c_size, c_ptr]),
    "gnn_gemm_nt_planes_ok": (ctypes.c_int, [ctypes.POINTER(GnnGemmNTParams)]),
    "gnn_gemm_nt_colsum_blocks": (ctypes.c_int, [ctypes.POINTER(GnnGemmNTParams), ctypes.POINTER(c_i32)]),
    "gnn_colsum_finish_f32": (ctypes.c_int, [c_ptr, c_i32, c_i64, c_ptr, c_ptr]),
    "gnn_gemm_tn_planes_ok": (ctypes.c_int, [ctypes.POINTER(GnnGemmTNParams)]),
    "gnn_colsum_workspace_size": (ctypes.c_int, [c_i64, c_i64, ctypes.POINTER(c_size)]),
    "gnn_colsum_f32": (ctypes.c_int, [c_i64, c_i64, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr]),
    "gnn_masked_ce_workspace_size": (ctypes.c_int, [c_i64, ctypes.POINTER(c_size)]),
    "gnn_masked_ce_f32": (
        ctypes.c_int,
        [c_i64, c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_gcn_out_ce_f32": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i32, c_ptr, c_ptr, c_i64, c_ptr, c_ptr, c_ptr,
         ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_masked_ce_colsum_f32": (
        ctypes.c_int,
        [c_i64, c_i32, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, ctypes.c_float, c_ptr, c_i64, c_ptr, c_ptr, c_size, c_ptr,
         c_ptr],
    ),
    "gnn_clip_adam_workspace_size": (ctypes.c_int, [ctypes.POINTER(c_size)]),
    "gnn_neighbor_sample_workspace_size": (ctypes.c_int, [c_i64, c_i64, c_i64, ctypes.POINTER(c_size)]),
    "gnn_neighbor_sample": (
        ctypes.c_int,
        [ctypes.POINTER(GnnGraph), c_ptr, c_ptr, c_i64, c_i32, c_ptr, ctypes.c_uint64, c_ptr, c_i64, c_ptr, c_ptr,
         c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_clip_adam_f32": (ctypes.c_int, [ctypes.POINTER(GnnAdamGroup), c_ptr, c_ptr, c_ptr, c_size, c_ptr]),
    "gnn_bn_workspace_size": (ctypes.c_int, [c_i64, ctypes.POINTER(c_size)]),
    "gnn_bn_stats_f32": (
        ctypes.c_int,
        [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i32, ctypes.c_float, ctypes.c_float, c_ptr, c_ptr, c_ptr, c_ptr,
         c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_bn_finalize_f32": (
        ctypes.c_int, [c_ptr, c_i64, ctypes.c_float, ctypes.c_float, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr],
    ),
    "gnn_bn_act_res_fwd_f32": (
        ctypes.c_int,
        [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, ctypes.c_float, ctypes.c_uint64,
         c_ptr, c_ptr, c_i64, c_ptr],
    ),
    "gnn_bn_act_bwd_reduce_f32": (
        ctypes.c_int,
        [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, ctypes.c_float, ctypes.c_uint64,
         c_ptr, c_ptr, c_ptr, c_size, c_ptr],
    ),
    "gnn_bn_act_bwd_f32": (
        ctypes.c_int,
        [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, ctypes.c_float, ctypes.c_uint64,
         c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr],
    ),
    "gnn_bn_act_bwd_colsum_blocks": (ctypes.c_int, [c_i64, c_i64, ctypes.POINTER(c_i32)]),
    "gnn_bn_act_bwd_colsum_f32": (
        ctypes.c_int,
        [c_ptr, c_i64, c_ptr, c_i64, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, ctypes.c_float, ctypes.c_uint64,
         c_ptr, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr],
    ),
    "gnn_time_inject_sin_f32": (
        ctypes.c_int,
        [c_ptr, c_i64, c_i64, c_i64, c_ptr, c_i64, c_i64, c_ptr, c_i64, c_ptr],
    ),
}

_LIB: ctypes.CDLL | None = None


class GnnmpError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libgnnmp.so (once).  Raises if it is missing — there is no fallback path."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise GnnmpError(
            f"{LIB_PATH} not found: build it with `make -C {PKG_DIR / 'csrc'}` "
            "(or __graft_entry__.build()).  The MI355X kernels are required; there is no CPU fallback."
        )
    lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    ver = lib.gnn_abi_version()
    if ver != ABI_VERSION:
        raise GnnmpError(f"libgnnmp ABI {ver} != expected {ABI_VERSION}; rebuild the library")
    _LIB = lib
    return lib


def check(status: int, what: str = "") -> None:
    if status == GNN_OK:
        return
    lib = load()
    msg = lib.gnn_last_error().decode(errors="replace")
    kind = lib.gnn_status_string(status).decode()
    exc = _STATUS_EXC.get(status, GnnmpError)
    raise exc(f"libgnnmp {what or 'call'} failed ({kind}): {msg}")


def stream_handle(device: torch.device | None = None) -> int:
    """The caller's current HIP stream (torch.cuda.current_stream), as a raw pointer."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


CALLS = [0]  # libgnnmp calls made so far (distributed.GradBucket tells gradient producers apart by it)


def call(name: str, *args) -> None:
    lib = load()
    CALLS[0] += 1
    check(getattr(lib, name)(*args), name)
