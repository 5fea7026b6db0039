"""ctypes binding of the C-ABI library `libasrx.so` (include/asrx.h).

Loaded after `import torch` so that the library's libamdhip64.so.7 dependency resolves to the HIP runtime
torch already mapped (both carry SONAME libamdhip64.so.7).  There is NO fallback: if the library is
missing, every op raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must be imported first: binds the HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ASRX_LIB", os.path.join(_HERE, "lib", "libasrx.so"))

BF16 = 0
F32 = 1
BITS = 2  # gate operand only: 1 bit per element, uint32 words

c_i32, c_i64, c_u64, c_f32, c_vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float, ctypes.c_void_p


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ("m", c_i32), ("n", c_i32), ("k", c_i32),
        ("in_dtype", c_i32),
        ("a", c_vp), ("lda", c_i64), ("a_trans", c_i32),
        ("b", c_vp), ("ldb", c_i64), ("b_trans", c_i32),
        ("c", c_vp), ("ldc", c_i64), ("c_dtype", c_i32),
        ("batch", c_i32), ("batch_inner", c_i32),
        ("sa_outer", c_i64), ("sa_inner", c_i64), ("sb_outer", c_i64), ("sb_inner", c_i64),
        ("sc_outer", c_i64), ("sc_inner", c_i64),
        ("alpha", c_f32), ("beta", c_f32),
        ("bias", c_vp),
        ("rowadd", c_vp), ("ld_rowadd", c_i64), ("rowadd_mod", c_i32),
        ("relu", c_i32),
        ("dropout_p", c_f32), ("seed", c_u64),
        ("gate", c_vp), ("ld_gate", c_i64), ("gate_dtype", c_i32),
        ("resid", c_vp), ("ld_resid", c_i64), ("resid_dtype", c_i32),
        ("splitk", c_i32), ("workspace", c_vp), ("workspace_elems", c_i64),
        ("tile", c_i32),
        ("rowsum_a", c_vp), ("rowsum_ws", c_vp),
        ("mask_out", c_vp), ("ld_mask", c_i64),
        ("kernel", c_i32),
    ]


class GemmGroupDev(ctypes.Structure):
    """asrx_gemm_group_dev: one 64-byte entry of a grouped launch's device table."""
    _fields_ = [
        ("a", c_vp), ("b", c_vp), ("c", c_vp), ("rowsum_a", c_vp),
        ("lda", c_i32), ("ldb", c_i32), ("ldc", c_i32), ("m", c_i32), ("n", c_i32), ("k", c_i32),
        ("tile_start", c_i32), ("reserved", c_i32),
    ]


class RowsumGroup(ctypes.Structure):
    _fields_ = [("in_", c_vp), ("rows", c_i64), ("cols", c_i32), ("out", c_vp), ("accumulate", c_i32)]


MAX_ROWSUM_GROUPS = 64   # norm.hip RG_MAX


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ("batch", c_i32), ("heads", c_i32), ("lq", c_i32), ("lk", c_i32), ("dh", c_i32),
        ("q", c_vp), ("q_rstride", c_i64), ("q_bstride", c_i64),
        ("k", c_vp), ("k_rstride", c_i64), ("k_bstride", c_i64),
        ("v", c_vp), ("v_rstride", c_i64), ("v_bstride", c_i64),
        ("o", c_vp), ("o_rstride", c_i64), ("o_bstride", c_i64),
        ("lse", c_vp),
        ("scale", c_f32),
        ("mask_mode", c_i32), ("causal", c_i32),
        ("kvalid", c_vp), ("qvalid", c_vp), ("valid_bstride", c_i64),
        ("mask", c_vp), ("mask_sb", c_i64), ("mask_sq", c_i64), ("mask_sk", c_i64),
        ("dropout_p", c_f32), ("seed", c_u64),
        ("dout", c_vp), ("do_rstride", c_i64), ("do_bstride", c_i64),
        ("dq", c_vp), ("dq_rstride", c_i64), ("dq_bstride", c_i64),
        ("dk", c_vp), ("dk_rstride", c_i64), ("dk_bstride", c_i64),
        ("dv", c_vp), ("dv_rstride", c_i64), ("dv_bstride", c_i64),
        ("delta", c_vp), ("dq_acc", c_vp),
        ("dropmask", c_vp), ("dropmask_ready", c_i32),
        ("o_lo", c_vp),
    ]


class AdamDesc(ctypes.Structure):
    _fields_ = [
        ("p", c_vp), ("m", c_vp), ("v", c_vp), ("p_bf16", c_vp), ("g_base", c_vp), ("hyp", c_vp),
        ("lr", c_f32), ("beta1", c_f32), ("beta2", c_f32), ("eps", c_f32), ("weight_decay", c_f32),
        ("bias_corr1", c_f32), ("bias_corr2", c_f32), ("grad_scale", c_f32),
        ("decoupled", c_i32), ("reserved", c_i32),
    ]


# name -> argtypes (restype is int for all)
SIGNATURES = {
    "asrx_version": [],
    "asrx_struct_sizes": [ctypes.POINTER(c_i64), c_i32],
    "asrx_gemm": [ctypes.POINTER(GemmDesc), c_vp],
    "asrx_gemm_kernel_name": [ctypes.POINTER(GemmDesc), ctypes.c_char_p, c_i32],
    "asrx_gemm_set_debug": [c_i32],
    "asrx_set_tuning": [c_i32, c_i32],
    "asrx_gemm_grouped_xcd": [ctypes.POINTER(GemmDesc), c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "asrx_gemm_grouped_xcd_adam": [ctypes.POINTER(GemmDesc), c_vp, c_vp, c_vp, c_i32, c_i32, c_i32,
                                   ctypes.POINTER(AdamDesc), c_vp],
    "asrx_adam_spans": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32,
                        c_f32, c_i32, c_vp, c_vp],
    "asrx_reduce_rows_grouped": [ctypes.POINTER(RowsumGroup), c_i32, c_vp],
    "asrx_attention_fwd": [ctypes.POINTER(AttnDesc), c_vp],
    "asrx_attn_dropgen": [ctypes.POINTER(AttnDesc), c_vp],
    "asrx_layernorm_fwd_attn_dropgen": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32,
                                        ctypes.POINTER(AttnDesc), c_vp],
    "asrx_attention_bwd": [ctypes.POINTER(AttnDesc), c_vp],
    "asrx_attn_delta": [ctypes.POINTER(AttnDesc), c_vp],
    "asrx_softmax_fwd": [c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i32, c_i64, c_f32, c_i32, c_i32, c_vp, c_vp,
                         c_i64, c_vp, c_i64, c_i64, c_i64, c_f32, c_u64, c_vp],
    "asrx_softmax_bwd": [c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_i64, c_f32, c_f32, c_u64, c_vp],
    "asrx_layernorm_fwd": [c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_f32, c_vp],
    "asrx_layernorm_bwd": [c_i32, c_vp, c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_f32, c_u64, c_vp,
                           c_i32, c_i64, c_i32, c_vp],
    "asrx_reduce_rows": [c_i32, c_vp, c_i64, c_i32, c_i64, c_vp, c_i32, c_vp, c_i32, c_vp],
    "asrx_conv1_fwd": [c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i32, c_vp, c_vp],
    "asrx_im2col_conv2": [c_i32, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp],
    "asrx_conv2_fwd": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp],
    "asrx_conv_bwd_implicit": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp],
    "asrx_conv2_wgrad": [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp, c_vp, c_i64, c_vp, c_i32, c_vp],
    "asrx_col2im_conv2": [c_i32, c_vp, c_i32, c_vp, c_i32, c_i32, c_i32, c_vp, c_vp],
    "asrx_conv1_bwd_w": [c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp],
    "asrx_conv1_bwd_fused": [c_i32, c_vp, c_i32, c_vp, c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp, c_vp],
    "asrx_embed_fwd": [c_vp, c_i64, c_i32, c_vp, c_i32, c_vp, c_f32, c_u64, c_vp, c_vp],
    "asrx_embed_bwd": [c_vp, c_i64, c_i32, c_vp, c_i32, c_i32, c_i32, c_f32, c_u64, c_vp, c_vp],
    "asrx_cross_entropy": [c_vp, c_i64, c_i32, c_i64, c_vp, c_i64, c_f32, c_vp, c_vp, c_vp, c_vp, c_vp],
    "asrx_cast": [c_i32, c_vp, c_i32, c_vp, c_i64, c_vp],
    "asrx_ewise": [c_i32, c_i32, c_vp, c_i32, c_vp, c_i32, c_vp, c_i64, c_f32, c_u64, c_vp],
    "asrx_sum_chunks_bf16": [c_vp, c_i32, c_i64, c_vp, c_vp],
    "asrx_greedy_argmax": [c_vp, c_i64, c_i32, c_i64, c_vp, c_i64, c_vp, c_vp],
    "asrx_spectrogram": [c_vp, c_i64, c_i64, c_i64, c_vp, c_i32, c_i32, c_i32, c_i32, ctypes.c_float, c_vp, c_i64,
                         c_vp, c_vp],
    "asrx_adam": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32, c_i32,
                  c_vp, c_vp],
    "asrx_upload": [c_vp, c_vp, c_i64, c_vp],
    "asrx_set_seed_offset": [c_u64, c_vp],
    "asrx_dropout_mask": [c_vp, c_i64, c_f32, c_u64, c_vp],
    "asrx_zero_spans": [c_vp, c_vp, c_i32, c_vp],
    "asrx_clip_grad_norm": [c_vp, c_i32, c_f32, c_vp, c_i32, c_vp, c_vp],
    "asrx_remove_after_eos": [c_vp, c_i32, c_i32, c_vp, c_i32, c_i32, c_vp, c_i64, c_vp],
    "asrx_rowwise": [c_i32, c_vp, c_vp, c_vp, c_i64, c_i32, c_i64, c_vp],
    "asrx_transpose_last2": [c_vp, c_i64, c_i32, c_i32, c_vp, c_vp],
    "asrx_step_tokens": [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp, c_vp, c_vp],
}

ERRORS = {-1: "bad argument", -2: "launch failure", -3: "unsupported shape/layout"}

_lib = None


def lib():
    """Load (once) and return the ctypes library. Raises if the HIP library was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"asrx: native library not found at {LIB_PATH}; run __graft_entry__.build() "
                               f"(python -m asrx._build). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_int
        # size helper (host arithmetic, int64 result)
        L.asrx_attn_dropmask_words.argtypes = [c_i32, c_i32, c_i32, c_i32]
        L.asrx_attn_dropmask_words.restype = c_i64
        L.asrx_attn_dq_acc_elems.argtypes = [c_i32, c_i32, c_i32, c_i32, c_i32]
        L.asrx_attn_dq_acc_elems.restype = c_i64
        _lib = L
    return _lib


def check(rc, name):
    if rc != 0:
        raise RuntimeError(f"asrx: {name} failed: {ERRORS.get(rc, rc)}")


_FNS = {}


def call(name, *args):
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"asrx: {name} failed: {ERRORS.get(rc, rc)}")
