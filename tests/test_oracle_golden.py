"""The CPU oracle against the reference's own golden vectors (bit-exact).  CPU only."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import fake_quant_np as FQ
from oracle import fake_quant_torch as FT


def same_bits(a, b):
    a = np.ascontiguousarray(a, dtype=np.float16)
    b = np.ascontiguousarray(b, dtype=np.float16)
    return a.shape == b.shape and np.array_equal(a.view(np.uint16), b.view(np.uint16))


def _bits(key):
    return int(key.split("_b")[1].split("_")[0])


def test_weight_group_np(golden):
    g = golden["fake_quant_golden"]
    keys = [k[:-3] for k in g.files if k.startswith("wgroup") and k.endswith("_in")]
    assert len(keys) == 14
    for k in keys:
        gs = 0 if k.startswith("wgroup0") else 128
        assert same_bits(FQ.quantize_weight_absmax(g[k + "_in"], _bits(k), gs), g[k + "_out"]), k


def test_weight_torch_backend(golden):
    g = golden["fake_quant_golden"]
    for k in [k[:-3] for k in g.files if k.endswith("_in") and k.startswith(("wgroup", "wpc", "wpt"))]:
        w = torch.from_numpy(g[k + "_in"])
        if k.startswith("wgroup"):
            out = FT.weight_group(w, _bits(k), 0 if k.startswith("wgroup0") else 128)
        elif k.startswith("wpc"):
            out = FT.weight_per_channel(w, _bits(k))
        else:
            out = FT.weight_per_tensor(w, _bits(k))
        assert same_bits(out.numpy(), g[k + "_out"]), k


def test_weight_per_channel_and_tensor_np(golden):
    g = golden["fake_quant_golden"]
    for k in [k[:-3] for k in g.files if k.endswith("_in") and (k.startswith("wpc") or k.startswith("wpt"))]:
        fn = FQ.quantize_weight_per_channel_absmax if k.startswith("wpc") else FQ.quantize_weight_per_tensor_absmax
        assert same_bits(fn(g[k + "_in"], _bits(k)), g[k + "_out"]), k


@pytest.mark.parametrize("kind", ["atok", "achan", "aten", "agrp"])
def test_activation_np_and_torch(golden, kind):
    g = golden["fake_quant_golden"]
    keys = [k[:-3] for k in g.files if k.startswith(kind) and k.endswith("_in")]
    assert len(keys) == 3  # 4, 8, 16 bit
    for k in keys:
        b, x, want = _bits(k), g[k + "_in"], g[k + "_out"]
        if kind == "atok":
            got_np, got_t = FQ.quantize_activation_per_token_absmax(x, b), FT.per_token(torch.from_numpy(x), b)
        elif kind == "achan":
            got_np, got_t = FQ.quantize_activation_per_channel_absmax(x, b), FT.per_channel(torch.from_numpy(x), b)
        elif kind == "aten":
            got_np, got_t = FQ.quantize_activation_per_tensor_absmax(x, b), FT.per_tensor(torch.from_numpy(x), b)
        else:
            got_np = FQ.quantize_activation_per_channel_group_absmax(x, 8, b)
            got_t = FT.per_group(torch.from_numpy(x), 8, b)
        assert same_bits(got_np, want), k
        assert same_bits(got_t.numpy(), want), k


def test_zero_channel_16bit_is_nan_like_reference(golden):
    """A zero channel at 16 bit has scale half(1e-5/32767) = 0 -> 0/0 = NaN in the reference."""
    g = golden["fake_quant_golden"]
    out = g["achan_b16_out"]
    assert np.isnan(out[1, 3]).all()


def test_codes_reproduce_dequantized(golden):
    g = golden["fake_quant_golden"]
    for bits in (4, 8):
        w = g[f"wgroup_b{bits}_k320_in"]
        codes, scales, gsz = FQ.quantize_weight_absmax_codes(w, bits, 128)
        assert gsz == 64  # 320 % 128 != 0 -> 96 -> 64 (fake_quant.py:33-37)
        assert np.abs(codes).max() <= 2 ** (bits - 1) - 1
        dq = (codes.reshape(-1, gsz).astype(np.float32) * scales.reshape(-1, 1).astype(np.float32)).astype(np.float16)
        want = g[f"wgroup_b{bits}_k320_out"]
        # value-exact: integer codes cannot carry the sign of a rounded-to-zero weight, so the
        # reference's -0.0 comes back as +0.0 (equal as numbers; no effect on any dot product)
        assert np.array_equal(dq.reshape(w.shape), want)
        neg_zero = (want == 0) & np.signbit(want)
        assert same_bits(np.where(neg_zero, want, dq.reshape(w.shape)), want)


def test_shrink_rule():
    assert FQ.shrink_group(320, 128) == 64
    assert FQ.shrink_group(768, 128) == 128
    assert FQ.shrink_group(640, 128) == 128
    with pytest.raises(ZeroDivisionError):
        FQ.shrink_group(36, 128)
    assert FQ.per_group_size(12, 12, 8) == 6


def test_pseudo_quantize(golden):
    g = golden["fake_quant_golden"]
    for zp in (1, 0):
        o, s, z = FQ.pseudo_quantize_tensor(g[f"pqt_zp{zp}_in"], 4, 128, bool(zp))
        assert same_bits(o, g[f"pqt_zp{zp}_out"])
        assert same_bits(s, g[f"pqt_zp{zp}_scales"])
        if zp:
            assert same_bits(z, g[f"pqt_zp{zp}_zeros"])


def test_module_forwards_cpu(golden):
    """WxAxLinear / WxAxConv2d forward = F.linear / F.conv2d on the oracle-quantized weights
    (+ oracle act quant), exactly the reference's CPU computation."""
    g = golden["fake_quant_golden"]
    for bits in (4, 8):
        for qo in (0, 1):
            k = f"lin_w{bits}_qo{qo}"
            wq = FQ.quantize_weight_absmax(g[k + "_w"], bits, 128)
            assert same_bits(wq, g[k + "_wq"]), k
            y = F.linear(torch.from_numpy(g[k + "_x"]), torch.from_numpy(wq), torch.from_numpy(g[k + "_b"]))
            if qo:
                y = FT.per_token(y, 8)
            assert same_bits(y.numpy(), g[k + "_y"]), k
    for k in [k[:-2] for k in g.files if k.startswith("conv_") and k.endswith("_x")]:
        wq = FQ.quantize_weight_per_channel_absmax(g[k + "_w"], 8)
        assert same_bits(wq, g[k + "_wq"]), k
        stride = int(k.split("s")[-1].split("p")[0])
        pad = int(k.split("p")[-1].split("_")[0])
        qo = k.endswith("qo1")
        x = torch.from_numpy(g[k + "_x"])
        if qo:
            x = FT.per_channel(x, 8)
        y = F.conv2d(x, torch.from_numpy(wq), torch.from_numpy(g[k + "_b"]), stride, pad)
        if qo:
            y = FT.per_channel(y, 8)
        assert same_bits(y.numpy(), g[k + "_y"]), k


def test_smooth_fold(golden):
    s = golden["smooth_golden"]
    sc = FQ.smooth_scales(s["act"], [s[f"fc{i}_w_in"] for i in range(3)], 0.8)
    f32 = np.float32
    assert same_bits((s["ln_w_in"].astype(f32) / sc.astype(f32)).astype(np.float16), s["ln_w_out"])
    assert same_bits((s["ln_b_in"].astype(f32) / sc.astype(f32)).astype(np.float16), s["ln_b_out"])
    for i in range(3):
        assert same_bits((s[f"fc{i}_w_in"].astype(f32) * sc.astype(f32)[None]).astype(np.float16),
                         s[f"fc{i}_w_out"])
    assert same_bits(np.abs(s["hook_x"].reshape(-1, 320)).max(0), s["hook_amax"])


def test_install_decisions(golden):
    """The oracle's per-layer swap decisions and quantized buffers equal the reference's
    _apply_quant_fake_act on the same tree (quantizer.py:491-533)."""
    from oracle.unet_ref import quantize_state_dict
    g = golden["install_golden"]
    for tag, qc in (("w8a8qa1", dict(w_bit=8, a_bit=8, quantize_act=True)),
                    ("w4a16qa0", dict(w_bit=4, a_bit=16, quantize_act=False))):
        orig = {k.split("|", 1)[1]: torch.from_numpy(g[k]) for k in g.files if k.startswith(tag + "_orig|")}
        qsd, flags = quantize_state_dict(orig, dict(qc, q_group_size=128))
        qsd_np, _ = quantize_state_dict(orig, dict(qc, q_group_size=128), backend="numpy")
        for key in qsd:
            assert same_bits(qsd[key].numpy(), qsd_np[key].numpy()), key
        layers = {row.split("|")[0]: row.split("|") for row in g[tag + "_layers"]}
        assert set(layers) == set(flags)
        for name, (_, kind, oq) in layers.items():
            f = flags[name]
            assert kind == ("WxAxLinear" if f["kind"] == "linear" else "WxAxConv2d")
            if f["kind"] == "linear":
                assert (oq != "None") == f["out_quant"], name
            else:
                assert (oq != "None") == f["quant"], name
        for k in g.files:
            if k.startswith(tag + "_quant|"):
                key = k.split("|", 1)[1]
                assert same_bits(qsd[key].numpy(), g[k]), key


def test_awq_pack_oracle_and_export_vs_reference_golden():
    """The reference's own AWQ int4 packing (tests/golden/awq_pack_golden.npz): the oracle's
    unpack / dequantize restatement reproduces it, and this build's exporter writes the same words
    the reference's pack (AWQ_PACK_ORDER, column direction) writes; round trip through the AWQ order."""
    import os
    from oracle import awq_pack as AP
    from qdiff import export as E
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "awq_pack_golden.npz"))
    iw = AP.reverse_awq_order(AP.unpack_awq(g["qweight"]))
    assert np.array_equal(iw, g["iweight"]) and np.array_equal(iw, g["unpacked_iweight"])
    deq = AP.dequantize_gemm(g["qweight"], g["qzeros"], g["scales"], 128)
    assert np.array_equal(deq.view(np.uint16), g["dequantize_gemm"].view(np.uint16))
    assert np.array_equal(E._pack_cols(torch.from_numpy(g["iweight"])).numpy(), g["qweight"])
    assert np.array_equal(E._pack_cols(torch.from_numpy(g["izeros"])).numpy(), g["qzeros"])
    assert np.array_equal(E._unpack_cols(torch.from_numpy(g["qweight"])).numpy(), g["iweight"])
    # symmetric codes -> AWQ (zero 8) -> reference dequantize == half(q * s)
    rng = np.random.default_rng(3)
    codes = torch.from_numpy(rng.integers(-8, 8, (64, 256)).astype(np.int8))
    sc = torch.from_numpy((rng.random((64, 2)) * 0.05 + 1e-3).astype(np.float16))
    d = E.awq_pack_linear(codes, sc, 128)
    deq = AP.dequantize_gemm(d["qweight"].numpy(), d["qzeros"].numpy(), d["scales"].numpy(), 128)
    ref = (codes.float() * sc.float().repeat_interleave(128, 1)).half().numpy()
    assert np.array_equal(deq.T.view(np.uint16), ref.view(np.uint16))
    c2, s2 = E.awq_unpack_linear(d["qweight"], d["qzeros"], d["scales"], 128)
    assert torch.equal(c2, codes) and torch.equal(s2, sc)
