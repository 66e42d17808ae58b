"""ctypes binding of libqdiff.so (the C ABI declared in include/qdiff.h).

The library is built in-tree (``csrc/Makefile`` -> ``libqdiff.so`` next to this file).  There is
no fallback: if the library is missing or fails to load, every op raises ``RuntimeError``.
torch is imported (and its HIP runtime loaded) before the library so that libqdiff resolves
``libamdhip64.so.7`` to the runtime torch already uses: one HIP runtime, one set of streams.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libqdiff.so")
# A/B timing of two builds on one box (scripts/ab.sh) points this at a second in-tree build
LIB_PATH = os.environ.get("QD_LIB_PATH", LIB_PATH)

P = ctypes.c_void_p
I = ctypes.c_int
I64 = ctypes.c_int64
F = ctypes.c_float

# name -> argtypes (all return int status)
SIGNATURES = {
    "qd_version": [],
    "qd_device_arch": [ctypes.c_char_p, I],
    "qd_fill_zero": [P, ctypes.c_long, P],
    "qd_act_absmax": [P, I, I, I, I, I, I, I, P, P],
    "qd_act_fakequant": [P, P, I, I, I, I, I, I, I, I, P, P],
    "qd_act_apply": [P, P, I, I, I, I, I, I, I, I, P, P],
    "qd_act_quant_cat_nhwc": [P, I, P, I, I, I, I, P, I, P, P],
    "qd_act_apply_cat_nhwc": [P, I, P, I, I, I, I, P, P, P],
    "qd_act_fq_small_nhwc": [P, P, I, I, I, I, I, P],
    "qd_weight_quant": [P, I, I, I, I, P, P, P, P],
    "qd_pack_int4": [P, I, I, P, P],
    "qd_conv_weight_khwc": [P, I, I, I, I, I, P, P],
    "qd_linear_fwd": [P, I, I, I, P, I, P, P, I, P, P, P, I, I, I, P, I, P, ctypes.c_long, P],
    "qd_conv2d_fwd": [P, I, I, I, I, I, P, I, I, I, I, I, I, P, P, P, I, P, P, ctypes.c_long, P],
    "qd_conv2d_fq": [P, I, I, I, I, I, P, I, I, I, I, I, I, P, I, P, P, I, P, I, P, P, P, ctypes.c_long, P],
    "qd_fq_finalize": [P, P, I, I, I, I, P, P, I, P, P],
    "qd_colmax_geom_force": [I, I],
    "qd_attn_force": [I],
    "qd_groupnorm": [P, P, I, I, I, I, I, F, P, P, I, I, P, P, P],
    "qd_groupnorm_xamax": [P, P, I, I, I, I, I, F, P, P, I, I, P, P, P, P],
    "qd_groupnorm_fq_in": [P, P, I, P, I, I, I, I, I, F, P, P, I, I, P, P, P],
    "qd_groupnorm_fin": [P, P, I, P, P, I, P, I, I, I, I, F, P, P, I, I, P, P, P],
    "qd_layernorm": [P, I, I, F, P, P, P, P],
    "qd_layernorm_fq": [P, P, I, I, I, I, F, P, P, P, P, P],
    "qd_geglu": [P, I, I, P, P],
    "qd_silu": [P, P, I64, P],
    "qd_add": [P, P, P, I64, P],
    "qd_concat_c": [P, I, P, I, I64, P, P],
    "qd_nchw_to_nhwc": [P, I, I, I, I, P, P],
    "qd_nhwc_to_nchw": [P, I, I, I, I, P, P],
    "qd_attention": [P, I, P, I, P, I, P, I, I, I, I, I, I, F, P],
    "qd_attention_causal": [P, I, P, I, P, I, P, I, I, I, I, I, F, P],
    "qd_quant_rows_fp8": [P, ctypes.c_long, I, I, P, I, P, P],
    "qd_fp8_weight": [P, P, I, I, I, P, P, P],
    "qd_linear_fp8": [P, P, I, I, I, P, P, P, P, P, I, I, I, P],
    "qd_embed_tokens": [P, I64, I, P, I64, P, I, P, P],
    "qd_clip_act": [P, P, I64, I, P],
    "qd_gather_rows": [P, I64, I64, P, I, I, P, P],
    "qd_vae_prescale": [P, I64, I, I, F, F, I, I, P, P],
    "qd_vae_postprocess": [P, I, I64, I, I, P, P, P],
    "qd_timestep_embedding": [P, P, I, I, I, F, P, P],
    "qd_cfg_ddim_step": [P, P, I, I64, F, P, P, P, P, I, I, P],
    "qd_cfg_pndm_step": [P, P, I, I64, F, P, P, P, P, P, P, I, I, P],
    "qd_cfg_euler_discrete_step": [P, P, I, I64, F, P, P, P, P, I, I, P],
    "qd_scale_latents": [P, I64, F, F, P, I, I, P],
    "qd_channel_absmax_accum": [P, I64, I, P, P, P, P],
    "qd_smooth_fold": [P, P, P, P, I, I, P, F, P, P, P],
    "qd_gemm_force": [I],
    "qd_gemm_epi_lds": [I],
    "qd_gn_geom_force": [I, I],
    "qd_selftest_recip": [P, P],
    "qd_adaln_modulate": [P, I64, I, I, F, P, P, I, P, P],
    "qd_gated_residual": [P, P, I, P, I, I64, I, I, P, P],
    "qd_rmsnorm_heads": [P, I64, I, I, I, I64, I64, P, F, P],
    "qd_gelu_tanh": [P, P, I64, P],
    "qd_add_pos": [P, P, I, I64, I, P, P],
    "qd_copy_rows": [P, I, P, I, I64, I, I64, I64, P],
    "qd_unpatchify": [P, I, I, I, I, I, P, P],
    "qd_cfg_euler_step": [P, P, I, I64, F, P, P, P, P],
    "qd_quant_rows_i8": [P, ctypes.c_long, I, I, P, I, P, P],
    "qd_quant_samples_i8": [P, I, ctypes.c_long, P, P, P, I, P],
    "qd_quant_samples_i8_amax": [P, I, ctypes.c_long, P, I, P, P, P],
    "qd_linear_i8": [P, P, I, I, I, P, P, P, P, P, I, I, I, P, I, P, ctypes.c_long, P],
    "qd_linear_ln": [P, I, I, I, P, I, P, P, I, P, P, P, I, I, I, P, P, F, P, P, P, P, ctypes.c_long, P],
    "qd_linear_i8_ln": [P, P, I, I, I, P, P, P, P, P, I, I, I, P, P, F, P, P, P, P],
    "qd_linear_i8_geglu_q_ok": [I, I],
    "qd_linear_i8_geglu_q": [P, P, I, I, I, P, P, P, I, P, I, P, P],
    "qd_linear_ln_ok": [I],
    "qd_conv2d_i8": [P, P, I, I, I, I, I, P, P, I, I, I, I, I, I, P, P, P, I, P, P, I, P, P, ctypes.c_long, P],
    "qd_groupnorm_part": [P, P, P, P, I, I, I, I, I, F, P, P, I, P, P, P, P, P, P],
    "qd_quant_samples_i8_cat": [P, P, I, I, I, ctypes.c_long, P, P, P, P],
    "qd_groupnorm_i8": [P, P, I, P, I, P, I, I, I, I, I, F, P, P, I, P, P, P, P],
    "qd_layernorm_i8": [P, I, I, F, P, P, P, P, P],
}

# size queries (no status code)
QUERIES = {
    "qd_gemm_workspace": ([I, I, I, I, I, I, I], ctypes.c_long),
    "qd_groupnorm_workspace": ([I, I, I, I], I),
    "qd_gemm_i8_workspace": ([I, I, I, I, I], ctypes.c_long),
    "qd_act_fq_small_ok": ([I, I], I),
}

_lib = None
_load_error = None


def load():
    """Load libqdiff.so once; raise RuntimeError (never fall back) if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise RuntimeError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"libqdiff.so not found at {LIB_PATH}; build it with "
                       "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        raise RuntimeError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        _load_error = f"failed to load {LIB_PATH}: {e}"
        raise RuntimeError(_load_error) from e
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = I
    for name, (argtypes, restype) in QUERIES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    lib.qd_last_error.argtypes = []
    lib.qd_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


def call(name, *args):
    """Invoke an ``int``-returning entry point; non-zero status -> RuntimeError."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.qd_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (status {rc}): {msg}")
    return rc


def exported_symbols():
    return list(SIGNATURES) + list(QUERIES) + ["qd_last_error"]
