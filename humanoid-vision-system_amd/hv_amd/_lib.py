"""ctypes binding of libhvs.so (the C ABI declared in include/hv_kernels.h).

The library is built in-tree (``make -C humanoid-vision-system_amd``) and loaded after
torch so that it shares torch's HIP runtime (both carry the soname libamdhip64.so.7).
There is no fallback: if the library is missing every op raises.
"""
from __future__ import annotations

import ctypes as C
import glob
import hashlib
import os
import threading

import torch  # noqa: F401  (must be loaded first: HIP runtime shared by soname)

HV_F32, HV_BF16 = 0, 1
# per-call kernel variants (include/hv_kernels.h HV_GV_* / HV_MV_*): 0 = automatic
GV_TILE_128x128, GV_TILE_64x128, GV_TILE_128x64, GV_TILE_64x64, GV_TILE_256, GV_TILE_SMALLK = 1, 2, 3, 4, 5, 6
GV_REGSTAGE, GV_NO_BIG, GV_BIG_ALWAYS, GV_NO_SMALL = 0x8, 0x10, 0x20, 0x40
GV_TRAIN128, GV_FLAT_EPI, GV_FLAT_TRAIN, GV_SHALLOW = 0x80, 0x100, 0x200, 0x400
GV_CONV_KTAIL, GV_NO_SMALLK, GV_SK_DIAG1, GV_SK_DIAG2 = 0x800, 0x1000, 0x2000, 0x4000
GV_SK_RES3, GV_SK_RES4, GV_TRAIN_BIG, GV_DEEP8, GV_NO_DEEP8 = 0x8000, 0x10000, 0x20000, 0x40000, 0x80000
GV_TRAIN_NOPF = 0x100000
MV_THREE_GROUPS, MV_ONE_GROUP8, MV_PERWAVE128, MV_PERWAVE64, MV_WIDE, MV_ABLATE_SHIFT = 1, 2, 5, 6, 0x100, 16
MV_SPLIT256, MV_SPLITW = 0x200, 12
MV_NOMERGE, MV_PIPE, MV_PIPE_NOMERGE, MV_PERWAVE = 7, 8, 9, 10
MV_TOK, MV_TOK16 = 0x400, 0x800
MV_TOKSPLIT2, MV_TOKSPLIT4 = 0x1000, 0x2000
ACT = {"none": 0, "relu": 1, "silu": 2, "gelu": 3, "leaky": 4, "sigmoid": 5}

ABI_VERSION = 4          # include/hv_kernels.h HV_ABI_VERSION this binding is written against
_LIB = None
_LOCK = threading.Lock()
_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HV_LIB_PATH: load another build of the same C ABI (A/B of two builds in one GPU call)
LIB_PATH = os.environ.get("HV_LIB_PATH") or os.path.join(_PKG, "hv_amd", "libhvs.so")


def source_hash() -> str | None:
    """The Makefile's HV_SRC_HASH recomputed from the sources in this tree (None when they are
    absent): sha256 over the sorted csrc/*.hip, csrc/*.h, ../include/*.h, then the Makefile."""
    files = sorted(glob.glob("csrc/*.hip", root_dir=_PKG) + glob.glob("csrc/*.h", root_dir=_PKG) +
                   glob.glob("../include/*.h", root_dir=_PKG)) + ["Makefile"]
    h = hashlib.sha256()
    for f in files:
        p = os.path.join(_PKG, f)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id() -> str:
    return lib().hv_build_id().decode()

vp = C.c_void_p
i32 = C.c_int
i64 = C.c_long
f32 = C.c_float


class SinkhornEntry(C.Structure):
    _fields_ = [("raw", vp), ("out", vp), ("history", vp), ("work", vp),
                ("batch", i32), ("n", i32), ("m", i32), ("iters", i32),
                ("eps", f32), ("tau", f32),
                ("row_block_start", i32), ("col_start", i32), ("row_start", i32), ("pad_", i32)]


class GemmDesc(C.Structure):
    _fields_ = [("dtype", i32), ("M", i32), ("N", i32), ("K", i32),
                ("A", vp), ("lda", i64),
                ("A2", vp), ("lda2", i64), ("k1", i32),
                ("B", vp), ("ldb", i64),
                ("C", vp), ("ldc", i64), ("c_dtype", i32),
                ("a_mean", vp), ("a_rstd", vp),
                ("scale", vp), ("bias", vp),
                ("act", i32), ("alpha", f32),
                ("residual", vp), ("ldr", i64), ("r_dtype", i32), ("r_mod", i32),
                ("conv_n", i32), ("conv_h", i32), ("conv_w", i32), ("conv_c", i32),
                ("conv_k", i32), ("conv_stride", i32), ("conv_pad", i32),
                ("conv_oh", i32), ("conv_ow", i32), ("b_colsum", vp),
                ("aux", vp), ("ld_aux", i64), ("aux_dtype", i32), ("epi_mode", i32),
                ("drop_p", f32), ("drop_seed", C.c_uint), ("conv_transposed", i32), ("variant", i32),
                ("splitk_work", vp), ("splitk_count", vp), ("splitk", i32), ("pad2_", i32),
                ("seed_offset", vp), ("colsum_part", vp)]


class CopySegment(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("bytes", C.c_longlong)]


class WgradDesc(C.Structure):
    _fields_ = [("dtype", i32), ("P", i32), ("N1", i32), ("N2", i32),
                ("A", vp), ("lda", i64), ("B", vp), ("ldb", i64), ("C", vp), ("ldc", i64),
                ("accumulate", i32), ("variant", i32), ("work", vp),
                ("conv_n", i32), ("conv_h", i32), ("conv_w", i32), ("conv_c", i32),
                ("conv_k", i32), ("conv_stride", i32), ("conv_pad", i32),
                ("conv_oh", i32), ("conv_ow", i32), ("pad2_", i32)]


class SinkhornBwdEntry(C.Structure):
    _fields_ = [("fwd", SinkhornEntry), ("dout", vp), ("draw", vp), ("bwork", vp)]


class NmsScale(C.Structure):
    _fields_ = [("boxes", vp), ("class_scores", vp), ("class_indices", vp), ("cells", i64)]


class ParamEntry(C.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp),
                ("n", i64), ("group", i32), ("blk", i32)]


class MhcFusedArgs(C.Structure):
    _fields_ = [("dtype", i32), ("D", i32), ("Hd", i32), ("T", i32),
                ("x", vp), ("a1t", vp), ("c1", vp), ("w2", vp), ("b2", vp), ("wct", vp),
                ("g_post", vp), ("b_post", vp), ("residual", vp), ("out", vp), ("variant", i32), ("pad_", i32),
                ("split_work", vp), ("split_count", vp)]


class SymeigEntry(C.Structure):
    _fields_ = [("h", vp), ("eig", vp), ("work", vp), ("n", i32), ("row_start", i32)]


class MhcPrepEntry(C.Structure):
    _fields_ = [("h_pre_raw", vp), ("h_post_raw", vp), ("h_res", vp), ("gamma_pre", vp), ("beta_pre", vp),
                ("w1", vp), ("b1", vp), ("a1", vp), ("c1", vp), ("wct", vp), ("scratch", vp), ("cs", vp),
                ("D", i32), ("Hd", i32), ("fold", i32), ("pad_", i32), ("blk", i32 * 4)]


class TransposeEntry(C.Structure):
    _fields_ = [("x", vp), ("y", vp), ("rows", i32), ("cols", i32), ("x_dtype", i32), ("y_dtype", i32),
                ("transpose", i32), ("blk", i32)]


class WprepEntry(C.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("gamma", vp), ("beta", vp), ("mean", vp), ("var", vp),
                ("cbias", vp), ("scale_out", vp), ("bias_out", vp), ("n", i64),
                ("kind", i32), ("dtype", i32), ("cin", i32), ("k", i32), ("ldk", i32), ("blk", i32),
                ("eps", f32), ("pad_", i32)]


_SIGS = {
    "hv_mhc_prep_scratch_floats": ([i32, i32], C.c_size_t),
    "hv_mhc_prep_blocks": ([i32, i32, i32, vp], None),
    "hv_mhc_prep_group": ([vp, i32, i32, vp, vp], i32),
    "hv_wprep_blocks": ([i32, i64, i32, i32], i32),
    "hv_wprep_group": ([vp, i32, i32, vp], i32),
    "hv_mhc_fused_supported": ([i32, i32, i32, i32], i32),
    "hv_mhc_fused": ([vp, vp], i32),
    "hv_mhc_fused_group": ([vp, i32, vp], i32),
    "hv_transpose_blocks": ([i32, i32], i32),
    "hv_transpose_group": ([vp, i32, i32, vp], i32),
    "hv_diag_launch_counts": ([vp], None),
    "hv_diag_reset_counts": ([], None),
    "hv_abi_version": ([], i32),
    "hv_build_id": ([], C.c_char_p),
    "hv_struct_sizes": ([vp], None),
    "hv_symeig_work_doubles": ([i32], C.c_size_t),
    "hv_symeig_group": ([vp, vp, i32, vp], i32),
    "hv_stability_work_floats": ([i32], C.c_size_t),
    "hv_stability_stats": ([i32, vp, vp, i32, i32, vp, i32, vp, vp, i32, vp, vp], i32),
    "hv_sinkhorn_work_floats": ([i32, i32, i32, i32], C.c_size_t),
    "hv_sinkhorn_group_forward": ([vp, i32, i32, i32, i32, i32, vp], i32),
    "hv_sinkhorn_group_forward_part": ([vp, i32, i32, i32, i32, i32, i32, vp], i32),
    "hv_sinkhorn_small_max_iters": ([], i32),
    "hv_gemm": ([vp, vp], i32),
    "hv_row_stats": ([i32, vp, i64, i32, i32, f32, vp, vp, vp], i32),
    "hv_layernorm": ([i32, vp, i32, i32, f32, vp, vp, i32, vp, vp, i32, vp], i32),
    "hv_rmsnorm": ([i32, vp, i32, i32, f32, vp, vp, vp], i32),
    "hv_mhc_prep": ([i32, i32, vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp], i32),
    "hv_cast": ([vp, i64, i32, vp, vp], i32),
    "hv_gemv": ([vp, vp, vp, i32, i32, vp, vp], i32),
    "hv_conv_weight_prep": ([vp, i32, i32, i32, vp, i32, vp, vp], i32),
    "hv_bn_fold": ([i32, vp, vp, vp, vp, vp, f32, vp, vp, vp], i32),
    "hv_nchw_to_nhwc": ([vp, i32, i32, i32, i32, i32, vp, vp], i32),
    "hv_maxpool2x2": ([i32, vp, i32, i32, i32, i32, vp, vp], i32),
    "hv_scale_maxpool2x2": ([i32, vp, vp, i32, i32, i32, i32, vp, vp], i32),
    "hv_conv_stem": ([i32, vp, i32, i32, i32, i32, i32, i32, i32, i32, vp, i32, i32, vp, vp, i32, vp, vp], i32),
    "hv_channel_mean_work_floats": ([i32, i32, i32], C.c_size_t),
    "hv_channel_mean": ([i32, vp, i32, i32, i32, vp, vp, vp], i32),
    "hv_se_mlp": ([vp, i32, i32, i32, vp, vp, vp, vp, vp, vp], i32),
    "hv_se_mlp2": ([vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp], i32),
    "hv_se_gate": ([i32, vp, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "hv_scale_residual": ([i32, vp, vp, vp, i32, i32, i32, vp, vp], i32),
    "hv_upsample_add": ([i32, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp], i32),
    "hv_add_scaled": ([i32, vp, vp, i64, f32, vp, vp], i32),
    "hv_add_rowvec": ([i32, vp, vp, i32, i32, i32, vp, vp], i32),
    "hv_interp_linear": ([vp, i32, i32, i32, vp, vp], i32),
    "hv_vit_tokens": ([i32, vp, vp, vp, vp, i32, i32, i32, vp, vp], i32),
    "hv_attention": ([i32, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp], i32),
    "hv_attention_work_elems": ([i32, i32, i32, i32], C.c_size_t),
    "hv_attention_mfma": ([vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, vp], i32),
    "hv_gather_rows": ([i32, vp, i64, i32, i32, vp, vp], i32),
    "hv_copy_segments": ([vp, i32, vp], i32),
    "hv_write_bytes": ([vp, vp, C.c_longlong, vp], i32),
    "hv_attention_general": ([i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, f32, vp], i32),
    "hv_yolo_decode": ([i32, vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "hv_nms_work_bytes": ([i32, i32, i32, C.c_long], C.c_size_t),
    "hv_preprocess": ([vp, i32, i32, i32, i32, i32, i32, vp, i32, i32, vp, vp], i32),
    "hv_pil_table_ints": ([i32, i32, i32, i32], C.c_size_t),
    "hv_pil_resample_tables": ([i32, i32, i32, i32, vp], i32),
    "hv_preprocess_pil": ([vp, i32, i32, i32, i32, i32, i32, vp, vp, i32, i32, vp, vp], i32),
    "hv_nms": ([vp, i32, i32, f32, f32, i32, C.c_long, vp, vp, vp, vp, vp, vp], i32),
    "hv_sort_desc_exact_work_bytes": ([i32], C.c_size_t),
    "hv_sort_desc_exact": ([vp, i32, i32, vp, vp, vp], i32),
    # ---- training step
    "hv_wgrad_work_floats": ([i32, i32, i32, i32], C.c_size_t),
    "hv_wgrad": ([vp, vp], i32),
    "hv_dgrad_weight_prep": ([vp, i32, i32, i32, i32, i32, vp, vp], i32),
    "hv_transpose_cast": ([vp, i32, i32, i32, vp, vp], i32),
    "hv_conv_grad_reorder": ([vp, i32, i32, i32, vp, vp], i32),
    "hv_colsum_work_floats": ([i32, i32], C.c_size_t),
    "hv_colsum": ([i32, vp, i64, i32, i32, vp, i32, vp, vp], i32),
    "hv_colsum_final": ([vp, i32, i32, vp, i32, vp], i32),
    "hv_bn_work_floats": ([i32, i32], C.c_size_t),
    "hv_bn_stats": ([i32, vp, i32, i32, f32, f32, vp, vp, vp, vp, vp, vp], i32),
    "hv_bn_apply": ([i32, vp, i32, i32, vp, vp, vp, vp, i32, vp, vp], i32),
    "hv_bn_backward": ([i32, vp, vp, i32, i32, vp, vp, vp, vp, i32, vp, vp, vp, vp, vp], i32),
    "hv_rownorm_train": ([i32, i32, vp, i32, i32, f32, vp, vp, f32, C.c_uint, vp, i32, vp, vp, vp, vp, vp], i32),
    "hv_rownorm_work_floats": ([i32, i32], C.c_size_t),
    "hv_rownorm_backward": ([i32, i32, vp, i32, vp, i32, i32, vp, vp, vp, f32, C.c_uint, vp, i32, vp, vp, vp, vp,
                             vp, vp], i32),
    "hv_act_backward": ([i32, vp, vp, i64, i32, f32, C.c_uint, vp, vp, vp], i32),
    "hv_mhc_param_backward_work_floats": ([i32, i32], C.c_size_t),
    "hv_mhc_param_backward": ([i32, i32] + [vp] * 14 + [vp], i32),
    "hv_dropout": ([i32, vp, i64, f32, C.c_uint, vp, vp, vp], i32),
    "hv_sinkhorn_bwd_work_floats": ([i32, i32, i32], C.c_size_t),
    "hv_sinkhorn_group_backward": ([vp, i32, i32, i32, i32, i32, vp], i32),
    "hv_chan_dot_work_floats": ([i32, i32, i32], C.c_size_t),
    "hv_chan_dot": ([i32, vp, vp, i32, i32, i32, vp, vp, vp], i32),
    "hv_se_mlp_backward": ([vp, vp, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
    "hv_se_backward_apply": ([i32, vp, vp, vp, i32, i32, i32, vp, vp], i32),
    "hv_maxpool2x2_backward": ([i32, vp, vp, i32, i32, i32, i32, vp, vp], i32),
    "hv_upsample_backward": ([i32, vp, i32, i32, i32, i32, i32, i32, vp, vp], i32),
    "hv_vit_assemble": ([i32, vp, vp, vp, i32, i32, i32, vp, vp], i32),
    "hv_vit_assemble_backward": ([i32, vp, i32, i32, i32, vp, vp, vp, vp], i32),
    "hv_scatter_rows": ([i32, vp, i64, i32, i32, vp, vp], i32),
    "hv_attention_train": ([i32, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, C.c_uint, vp, vp], i32),
    "hv_attention_backward": ([i32, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, f32, f32, C.c_uint, vp, vp, vp, vp,
                               vp, vp], i32),
    "hv_attention_train_mfma_work_elems": ([i32, i32, i32], C.c_size_t),
    "hv_attention_train_mfma": ([vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, C.c_uint, vp, vp, vp], i32),
    "hv_attention_backward_mfma": ([vp, vp, vp, vp, vp, vp, i32, i32, i32, f32, f32, C.c_uint, vp, vp, vp, vp, vp,
                                    vp],
                                   i32),
    "hv_yolo_loss_work_floats": ([i32, i32, i32, i32], C.c_size_t),
    "hv_yolo_loss": ([i32, vp, vp, i32, i32, i32, i32, i32, f32, f32, f32, f32, vp, i32, vp, vp, vp], i32),
    "hv_param_blocks": ([i64], i32),
    "hv_grad_norms": ([vp, i32, i32, i32, vp, vp, vp, vp, vp, vp], i32),
    "hv_adamw": ([vp, i32, i32, vp, f32, f32, f32, f32, f32, i32, vp, vp, vp], i32),
    "hv_adamw_dev": ([vp, i32, i32, vp, vp, vp, vp, vp], i32),
}

EXPORTED = tuple(_SIGS)


def _declare(lib):
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    sizes = (C.c_int * 5)()
    lib.hv_struct_sizes(sizes)
    want = [C.sizeof(s) for s in (SinkhornEntry, GemmDesc, MhcFusedArgs, MhcPrepEntry, WprepEntry)]
    if list(sizes) != want:
        raise RuntimeError(f"libhvs struct layout mismatch: C {list(sizes)} vs ctypes {want}")


def lib():
    """Load (once) and return the HIP kernel library; raises if it is not built."""
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(
                        f"libhvs.so not found at {LIB_PATH}: build it with "
                        "`make -C humanoid-vision-system_amd` (there is no CPU fallback)")
                handle = C.CDLL(LIB_PATH)
                _declare(handle)
                if handle.hv_abi_version() != ABI_VERSION:
                    raise RuntimeError(f"libhvs ABI {handle.hv_abi_version()} != binding ABI {ABI_VERSION}")
                want = source_hash()
                got = handle.hv_build_id().decode()
                # the in-tree library must be built from exactly these sources (A/B builds loaded
                # through HV_LIB_PATH are older builds by design)
                if not os.environ.get("HV_LIB_PATH") and want is not None and got != want:
                    raise RuntimeError(
                        f"stale libhvs.so: built from sources {got}, tree has {want}; "
                        "rebuild with `make -C humanoid-vision-system_amd`")
                _LIB = handle
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        kind = {-1: "invalid argument", -2: "unsupported shape/layout"}.get(rc, f"hipError {rc}")
        raise RuntimeError(f"{what} failed: {kind}")


def dtype_code(t: torch.dtype) -> int:
    if t == torch.float32:
        return HV_F32
    if t == torch.bfloat16:
        return HV_BF16
    raise TypeError(f"unsupported activation dtype {t}")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
