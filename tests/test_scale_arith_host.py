"""The fake-quant scale's division by qmax as an f64 product (csrc/common.h fq_scale_rq, used by
fq_scales8): s = half(fp32(a / qmax)) must come out bit-identical when a / qmax is formed as
fp32(f64(a) * rq) with rq within 2^-50 (relative) of 1 / qmax, for every odd qmax.  The device's rq
comes from the hardware f64 reciprocal estimate and two Newton steps, so the check covers rq
perturbed by +-2^-50 as well as the correctly rounded reciprocal.  CPU only (numpy's fp32 division
is IEEE correctly rounded: the reference's torch-CPU scale, fake_quant.py:44-46)."""
import numpy as np
import pytest


def _amax_samples(rng, n):
    # amax >= half(1e-5) (the clamp), spread over the fp32 exponent range the scales see, with
    # mantissas at both ends of the binade and at random
    e = rng.integers(-16, 17, n).astype(np.float64)
    m = rng.random(n)
    m[: n // 8] = 0.0
    m[n // 8: n // 4] = 1.0 - 2.0 ** -23
    a = (np.ldexp(1.0 + m, e.astype(np.int64))).astype(np.float32)
    return np.maximum(a, np.float32(np.float16(1e-5)))


@pytest.mark.parametrize("qmax", [1, 3, 7, 15, 127, 255, 2047, 32767])
def test_scale_division_as_f64_product(qmax):
    rng = np.random.default_rng(qmax)
    a = _amax_samples(rng, 2_000_000)
    exact = (a / np.float32(qmax)).astype(np.float32)
    # every integer multiple of qmax-related grid points: a = k * qmax * 2^e (exact quotients)
    k = rng.integers(1, 1 << 16, 200_000).astype(np.float64)
    a2 = np.ldexp(k * qmax, rng.integers(-30, 0, k.size)).astype(np.float32)
    a2 = a2[np.isfinite(a2) & (a2 >= np.float32(np.float16(1e-5)))]
    exact2 = (a2 / np.float32(qmax)).astype(np.float32)
    for rel in (0.0, 2.0 ** -50, -(2.0 ** -50)):
        rq = (1.0 / qmax) * (1.0 + rel)
        for aa, ex in ((a, exact), (a2, exact2)):
            got = (aa.astype(np.float64) * rq).astype(np.float32)
            assert np.array_equal(got.view(np.uint32), ex.view(np.uint32)), (qmax, rel)
            assert np.array_equal(got.astype(np.float16).view(np.uint16), ex.astype(np.float16).view(np.uint16))
