"""Restatement of the reference's AWQ int4 unpack / dequantize (TEST INFRASTRUCTURE ONLY):
utils/packing_utils.py:8-40 (unpack_awq: columnwise 4-bit unpack of int32 words; reverse_awq_order
with AWQ_REVERSE_ORDER [0, 4, 1, 5, 2, 6, 3, 7]) and :80-102 (dequantize_gemm: (w - z) * s with the
group scales / zeros repeated over group_size input rows), pinned by tests/golden/awq_pack_golden.npz
(generated from the reference's own functions by tests/golden/make_awq_golden.py)."""
import numpy as np

AWQ_REVERSE_ORDER = [0, 4, 1, 5, 2, 6, 3, 7]


def unpack_awq(qweight):
    """int32 [R, C / 8] -> 4-bit values [R, C] in AWQ (interleaved) order."""
    q = np.asarray(qweight).astype(np.int64) & 0xFFFFFFFF
    shifts = np.arange(0, 32, 4)
    return ((q[:, :, None] >> shifts[None, None, :]) & 0xF).reshape(q.shape[0], -1).astype(np.int8)


def reverse_awq_order(iw):
    idx = np.arange(iw.shape[-1]).reshape(-1, 8)[:, AWQ_REVERSE_ORDER].reshape(-1)
    return iw[:, idx]


def dequantize_gemm(qweight, qzeros, scales, group_size):
    """-> fp16 [in_features, out_features]: ((w - z) * s) with numpy fp16 arithmetic like torch's
    int8 - int8 then * half (one rounding of the exact product)."""
    iw = reverse_awq_order(unpack_awq(qweight)).astype(np.int16)
    iz = reverse_awq_order(unpack_awq(qzeros)).astype(np.int16)
    s = np.asarray(scales, np.float16)
    diff = (iw - np.repeat(iz, group_size, axis=0)).astype(np.float32)
    return (diff * np.repeat(s, group_size, axis=0).astype(np.float32)).astype(np.float16)
