"""The two GEMM / conv epilogue forms give the same bits (round 5; the post-residual amax - ff.net.2's -
joined the direct form in round 6).

gemm.hip's shared epilogue stores either straight from the MFMA fragments (v_permlane16_swap pairs
-> 16-B stores; the default wherever the epilogue needs no row-complete / slot view of the tile) or
through the LDS C tile (qd_gemm_epi_lds(1), the earlier form).  Both apply the same per-element
arithmetic (half(acc + bias), GEGLU / GELU-tanh, + residual), so every kernel variant must give
identical outputs and identical per-(sample, column) amax buffers under either form - fp16, int4
and int8 operands, ragged M, every forced tile / halo / split variant of each shape.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _set_lds(on):
    from qdiff import _lib
    _lib.call("qd_gemm_epi_lds", 1 if on else 0)


def _both(fn):
    """fn() under the direct form and under the LDS form -> (direct outputs, LDS outputs)."""
    try:
        _set_lds(False)
        a = [t.clone() for t in fn()]
        _set_lds(True)
        b = [t.clone() for t in fn()]
    finally:
        _set_lds(False)
    torch.cuda.synchronize()
    return a, b


def _eq(a, b, what):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x.shape == y.shape, what
        if x.dtype == torch.float16:
            assert torch.equal(x.view(torch.int16), y.view(torch.int16)), what
        else:
            assert torch.equal(x, y), what


def _variants(fam):
    from qdiff import kernels as K
    if fam == "f16":
        return [None] + list(K.REG_VARIANTS) + list(K.DMA_VARIANTS)
    if fam == "i8":
        return [None] + list(K.I8_VARIANTS) + list(K.I8_PERSIST_VARIANTS)
    return [None] + [v for v in K.W4_VARIANTS if v < 300]


def _forced(v, fn):
    from qdiff import kernels as K
    K.force_gemm(v)
    try:
        return _both(fn)
    except RuntimeError:  # a variant the library rejects for this shape
        return None
    finally:
        K.force_gemm(None)


@pytest.mark.parametrize("epi", ["bias", "bias_res", "plain", "amax", "amax_post", "geglu", "gelu_tanh"])
@pytest.mark.parametrize("M,N,Kd", [(1000, 320, 320), (4096, 640, 640), (520, 1280, 2560), (8192, 320, 1280)])
def test_linear_f16_direct_equals_lds(epi, M, N, Kd):
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(M + N + Kd)
    x = torch.randn(M, Kd, generator=g).half().to(DEV)
    n2 = 2 * N if epi == "geglu" else N
    w = (torch.randn(n2, Kd, generator=g) / Kd ** 0.5).half().to(DEV)
    b = torch.randn(n2, generator=g).half().to(DEV)
    r = torch.randn(M, N, generator=g).half().to(DEV)
    amx = epi in ("amax", "amax_post")
    if amx and M % 1024:
        pytest.skip("the amax epilogue needs whole-sample 64-row wave tiles")
    rps = 1024  # amax rows per sample
    am = torch.zeros((M // rps) * N, dtype=torch.float32, device=DEV) if amx else None
    post = epi == "amax_post"  # (ff.net.2: the amax of the final output, residual added)

    def run():
        if am is not None:
            am.zero_()
        y = K.linear(x, w, "f16", bias=None if epi == "plain" else b,
                     residual=r if epi in ("bias_res", "amax_post") else None,
                     amax=am, rows_per_sample=rps if amx else 0, geglu=epi == "geglu",
                     gelu_tanh=epi == "gelu_tanh", amax_post=post)
        return [y] + ([am] if am is not None else [])
    n = 0
    for v in _variants("f16"):
        res = _forced(v, run)
        if res is None:
            continue
        _eq(res[0], res[1], f"linear f16 {epi} M{M} N{N} K{Kd} variant {v}")
        n += 1
    assert n > 3


@pytest.mark.parametrize("epi", ["bias", "bias_res", "amax_post", "geglu"])
@pytest.mark.parametrize("M,N,Kd", [(32768, 320, 320), (1000, 640, 640), (2048, 1280, 5120), (8192, 320, 1280)])
def test_linear_i8_direct_equals_lds(epi, M, N, Kd):
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(7 * M + N)
    x = torch.randn(M, Kd, generator=g).half().to(DEV)
    n2 = 2 * N if epi == "geglu" else N
    w = (torch.randn(n2, Kd, generator=g) / Kd ** 0.5).half().to(DEV)
    b = torch.randn(n2, generator=g).half().to(DEV)
    r = torch.randn(M, N, generator=g).half().to(DEV)
    xq, sa = K.quant_rows_i8(x)
    wq, sw16, _ = K.weight_quant(w, Kd, 8, want_dq=False)
    sw = sw16.float().view(-1).contiguous()

    post = epi == "amax_post"
    if post and M % 1024:
        pytest.skip("the amax epilogue needs whole-sample 64-row wave tiles")
    am = torch.zeros((M // 1024) * N, dtype=torch.float32, device=DEV) if post else None

    def run():
        if post:
            am.zero_()
            return [K.linear_i8(xq, sa, wq, sw, bias=b, residual=r, amax=am, rows_per_sample=1024, amax_post=True), am]
        return [K.linear_i8(xq, sa, wq, sw, bias=b, residual=r if epi == "bias_res" else None, geglu=epi == "geglu")]
    n = 0
    for v in _variants("i8"):
        res = _forced(v, run)
        if res is None:
            continue
        _eq(res[0], res[1], f"linear i8 {epi} M{M} N{N} K{Kd} variant {v}")
        n += 1
    assert n > 3


def test_linear_i4_direct_equals_lds():
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(3)
    M, N, Kd = 1000, 640, 1280
    x = torch.randn(M, Kd, generator=g).half().to(DEV)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).half().to(DEV)
    b = torch.randn(N, generator=g).half().to(DEV)
    codes, sc, _ = K.weight_quant(w, 128, 4, want_dq=False)
    packed = K.pack_int4(codes)

    def run():
        return [K.linear(x, packed, "i4", scales=sc, group=128, bias=b)]
    for v in _variants("i4"):
        res = _forced(v, run)
        if res is not None:
            _eq(res[0], res[1], f"linear i4 variant {v}")


@pytest.mark.parametrize("n,hw,ci,co,res", [(8, 32, 320, 320, False), (2, 64, 320, 320, False), (4, 16, 640, 1280, True),
                                            (3, 8, 1280, 1280, False)])
def test_conv_f16_amax_direct_equals_lds(n, hw, ci, co, res):
    from qdiff import kernels as K
    g = torch.Generator().manual_seed(n * hw + ci)
    x = torch.randn(n, hw, hw, ci, generator=g).half().to(DEV)
    w = (torch.randn(co, 3, 3, ci, generator=g) / (9 * ci) ** 0.5).half().to(DEV)
    b = torch.randn(co, generator=g).half().to(DEV)
    r = torch.randn(n, hw, hw, co, generator=g).half().to(DEV) if res else None
    am = torch.zeros(n * co, dtype=torch.float32, device=DEV)

    def run():
        am.zero_()
        y = K.conv2d_nhwc(x, w, ci, 1, 1, bias=b, residual=r, amax=None if res else am)
        return [y] + ([] if res else [am])
    cands = _variants("f16") + list(K.HALO_VARIANTS) + [202 + 1000 * s for s in (2, 3)]
    n_ok = 0
    for v in cands:
        out = _forced(v, run)
        if out is None:
            continue
        _eq(out[0], out[1], f"conv f16 n{n} hw{hw} {ci}->{co} variant {v}")
        n_ok += 1
    assert n_ok > 3
