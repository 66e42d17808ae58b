"""Generate golden vectors from the reference's own fake-quant / quantizer code.

Run ONCE in the build container (needs /root/reference, read-only):

    python tests/golden/make_golden.py

It imports /root/reference/quantize/{fake_quant,quantizer,quantizer_SQ}.py in place (stubbing
only absent imports, see _refload.py), feeds them seeded synthetic fp16 inputs and writes the
inputs and outputs as plain arrays to tests/golden/*.npz (numpy, no pickles).  Only those data
fixtures are committed; no reference source or bytecode enters the repository.

Fixtures
--------
fake_quant_golden.npz   SURVEY.md §8c items 1-4 and 6: weight quantizers (group / per_channel /
                        per_tensor), activation quantizers (per_token / per_channel /
                        per_group / per_tensor, 4/8/16 bit), WxAxLinear / WxAxConv2d forward,
                        AwqQuantizer.pseudo_quantize_tensor.
smooth_golden.npz       §8c item 5: SqQuantizer.smooth_ln_fcs on LayerNorm(320) + 3 Linears.
install_golden.npz      the diffusion-branch module swap (quantizer.py:491-533) on a small
                        module tree: which layers become WxAx modules, with which flags, and
                        their fp16 buffers.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refload  # noqa: E402

F16 = np.float16


def rnd(rng, shape, scale=1.0, outliers=0):
    x = rng.standard_normal(shape).astype(np.float32) * scale
    if outliers:
        flat = x.reshape(-1)
        idx = rng.choice(flat.size, outliers, replace=False)
        flat[idx] *= 20.0
    return x.astype(F16)


def t16(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def gen_fake_quant(ref, out):
    fq = ref.fake_quant
    rng = np.random.default_rng(1234)
    # 1. quantize_weight_absmax (group) for b in {4,8}, K in SD1.5 Linear in_features.
    for bits in (4, 8):
        for k in (320, 640, 768, 1280, 2560, 5120):
            w = rnd(rng, (8, k), 0.05, outliers=3)
            w[0, :64] = 0  # an all-zero group exercises clamp(1e-5)
            key = f"wgroup_b{bits}_k{k}"
            out[key + "_in"] = w
            out[key + "_out"] = fq.quantize_weight_absmax(
                t16(w).clone(), n_bits=bits, group_size=128, codeBookQuantInd=False).numpy()
        # group_size 0: one scale per row
        w = rnd(rng, (16, 96), 0.1)
        out[f"wgroup0_b{bits}_in"] = w
        out[f"wgroup0_b{bits}_out"] = fq.quantize_weight_absmax(
            t16(w).clone(), n_bits=bits, group_size=0, codeBookQuantInd=False).numpy()
    # 2. per-channel (last dim) on conv weights; per-tensor
    for bits in (4, 8):
        for shp in ((64, 32, 3, 3), (64, 32, 1, 1), (32, 48)):
            w = rnd(rng, shp, 0.05, outliers=2)
            key = f"wpc_b{bits}_{'x'.join(map(str, shp))}"
            out[key + "_in"] = w
            out[key + "_out"] = fq.quantize_weight_per_channel_absmax(t16(w), bits).numpy()
        w = rnd(rng, (64, 32, 3, 3), 0.05, outliers=2)
        out[f"wpt_b{bits}_in"] = w
        out[f"wpt_b{bits}_out"] = fq.quantize_weight_per_tensor_absmax(t16(w), bits).numpy()
    # 3. activation quantizers
    for bits in (4, 8, 16):
        x = rnd(rng, (2, 77, 320), 1.0, outliers=8)
        out[f"atok_b{bits}_in"] = x
        out[f"atok_b{bits}_out"] = fq.quantize_activation_per_token_absmax(t16(x), bits).numpy()
        x = rnd(rng, (2, 64, 16, 16), 2.0, outliers=8)
        x[1, 3] = 0  # zero channel -> clamp path
        out[f"achan_b{bits}_in"] = x
        out[f"achan_b{bits}_out"] = fq.quantize_activation_per_channel_absmax(t16(x), bits).numpy()
        x = rnd(rng, (2, 64, 16, 16), 2.0, outliers=8)
        out[f"aten_b{bits}_in"] = x
        out[f"aten_b{bits}_out"] = fq.quantize_activation_per_tensor_absmax(t16(x), bits).numpy()
        x = rnd(rng, (2, 8, 12, 12), 1.0, outliers=4)
        out[f"agrp_b{bits}_in"] = x
        # group 8 does not divide 12 -> shrinks to 6 (fake_quant.py:138-139)
        out[f"agrp_b{bits}_out"] = fq.quantize_activation_per_channel_group_absmax(
            t16(x), group_size=8, n_bits=bits).numpy()
    # 4. module forwards
    torch.manual_seed(0)
    for bits_w in (4, 8):
        for qo in (False, True):
            lin = torch.nn.Linear(320, 640, bias=True).half()
            with torch.no_grad():
                lin.weight.copy_(t16(rnd(rng, (640, 320), 0.05, outliers=4)))
                lin.bias.copy_(t16(rnd(rng, (640,), 0.1)))
            w_in = lin.weight.detach().numpy().copy()
            m = fq.WxAxLinear.from_float(lin, weight_quant="group", act_quant="per_token",
                                         quantize_output=qo, n_bits_W=bits_w, n_bits_A=8,
                                         group_size_W=128)
            x = rnd(rng, (2, 77, 320), 1.0, outliers=6)
            key = f"lin_w{bits_w}_qo{int(qo)}"
            out[key + "_w"] = w_in
            out[key + "_b"] = lin.bias.detach().numpy()
            out[key + "_wq"] = m.weight.numpy()
            out[key + "_x"] = x
            out[key + "_y"] = m(t16(x)).numpy()
    for (cin, cout, k, stride, pad) in ((16, 32, 3, 1, 1), (16, 32, 3, 2, 1), (32, 16, 1, 1, 0)):
        for qo in (False, True):
            conv = torch.nn.Conv2d(cin, cout, k, stride=stride, padding=pad, bias=True).half()
            with torch.no_grad():
                conv.weight.copy_(t16(rnd(rng, conv.weight.shape, 0.1, outliers=4)))
                conv.bias.copy_(t16(rnd(rng, (cout,), 0.1)))
            w_in = conv.weight.detach().numpy().copy()
            m = fq.WxAxConv2d.from_float(conv, weight_quant="per_channel", act_quant="per_channel",
                                         quantize_output=qo, n_bits_W=8, n_bits_A=8)
            x = rnd(rng, (2, cin, 12, 12), 1.0, outliers=6)
            key = f"conv_c{cin}x{cout}k{k}s{stride}p{pad}_qo{int(qo)}"
            out[key + "_w"] = w_in
            out[key + "_b"] = conv.bias.detach().numpy()
            out[key + "_wq"] = m.weight.numpy()
            out[key + "_x"] = x
            out[key + "_y"] = m(t16(x)).numpy()
    # 6. pseudo_quantize_tensor (LLM path; kept for surface completeness)
    AQ = ref.quantizer.AwqQuantizer
    for zp in (True, False):
        slf = types.SimpleNamespace(group_size=128, zero_point=zp)
        w = rnd(rng, (16, 256), 0.05, outliers=3)
        wq, s, z = AQ.pseudo_quantize_tensor(slf, t16(w).clone(), bitWidth=4)
        out[f"pqt_zp{int(zp)}_in"] = w
        out[f"pqt_zp{int(zp)}_out"] = wq.numpy()
        out[f"pqt_zp{int(zp)}_scales"] = s.numpy()
        if z is not None:
            out[f"pqt_zp{int(zp)}_zeros"] = z.numpy()


def gen_smooth(ref, out):
    rng = np.random.default_rng(77)
    SQ = ref.quantizer_SQ.SqQuantizer
    ln = torch.nn.LayerNorm(320).half()
    fcs = [torch.nn.Linear(320, 320, bias=False).half() for _ in range(3)]
    with torch.no_grad():
        ln.weight.copy_(t16((1 + 0.1 * rng.standard_normal(320)).astype(F16)))
        ln.bias.copy_(t16((0.1 * rng.standard_normal(320)).astype(F16)))
        for i, fc in enumerate(fcs):
            fc.weight.copy_(t16(rnd(rng, (320, 320), 0.05, outliers=5)))
    act = np.abs(rnd(rng, (320,), 2.0, outliers=4)).astype(F16)
    out["ln_w_in"] = ln.weight.detach().numpy().copy()
    out["ln_b_in"] = ln.bias.detach().numpy().copy()
    for i, fc in enumerate(fcs):
        out[f"fc{i}_w_in"] = fc.weight.detach().numpy().copy()
    out["act"] = act
    SQ.smooth_ln_fcs(None, ln, fcs, t16(act), alpha=0.80)
    out["ln_w_out"] = ln.weight.detach().numpy()
    out["ln_b_out"] = ln.bias.detach().numpy()
    for i, fc in enumerate(fcs):
        out[f"fc{i}_w_out"] = fc.weight.detach().numpy()
    # the hook's per-call reduction (calib_data.py:105-124) on one call
    hook = ref.calib_data.Mean_Max_Activation_Hook()
    x = rnd(rng, (2, 64, 320), 1.0, outliers=6)
    hook(None, (t16(x),), None)
    out["hook_x"] = x
    out["hook_amax"] = hook.max_scales[0].numpy()
    # the mean over calls (StableDiffusion1_x.py:104-112 mean_of_dict: torch.mean of the stacked
    # per-call fp16 maxima) for 3, 24 and 600 calls (600 = the reference's calibration: 12 pipeline
    # calls x 50 steps); magnitudes spread over ~2^14 so the fp32 sums round
    sd15 = _refload.load_sd15_adapter()
    for calls in (3, 24, 600):
        hook = ref.calib_data.Mean_Max_Activation_Hook()
        xs = []
        for i in range(calls):
            xi = (rng.standard_normal((1, 4, 320)) * np.exp(rng.standard_normal(320) * 2.5)).astype(F16)
            hook(None, (t16(xi),), None)
            xs.append(xi)
        out[f"mean{calls}_x"] = np.stack(xs)
        out[f"mean{calls}_mean"] = sd15.StableDiffusion1_x.mean_of_dict(None, hook.max_scales).numpy()


class _Tiny(torch.nn.Module):
    """A small tree with every layer kind/name the diffusion swap distinguishes.

    Linear in_features must be a multiple of 32: the group shrink of fake_quant.py:33-37
    otherwise reaches g=0 and raises ZeroDivisionError (recorded separately below).
    """

    def __init__(self):
        super().__init__()
        self.conv_in = torch.nn.Conv2d(4, 64, 3, padding=1)
        self.blk = torch.nn.Module()
        self.blk.to_q = torch.nn.Linear(64, 64, bias=False)
        self.blk.add_k_proj = torch.nn.Linear(64, 64, bias=True)   # name matches 'k_proj'
        self.blk.proj_in = torch.nn.Conv2d(64, 64, 1)
        self.blk.ff = torch.nn.Sequential(torch.nn.Linear(64, 96), torch.nn.GELU(), torch.nn.Linear(96, 64))
        self.norm = torch.nn.GroupNorm(2, 64)


def gen_install(ref, out):
    AQ = ref.quantizer.AwqQuantizer
    rng = np.random.default_rng(5)
    for w_bit, a_bit, qa in ((8, 8, True), (4, 16, False)):
        torch.manual_seed(3)
        net = _Tiny().half()
        with torch.no_grad():
            for name, p in net.named_parameters():
                p.copy_(t16(rnd(rng, tuple(p.shape), 0.2)))
        slf = types.SimpleNamespace(diffusion_model=True, weight_quant_type="group",
                                    weight_quant_conv_type="per_channel",
                                    act_quant_conv_type="per_channel",
                                    act_quant_conv_group_size=1, quantise_act=qa,
                                    a_bit=a_bit, group_size=128, codeBookQuantInd=False)
        orig = {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}
        trav = AQ.MyTraversal()
        for name, child in net.named_children():
            trav.traverse(name, child, net)
        AQ._apply_quant_fake_act(slf, net, trav.get_lin_conv(), w_bit, debugStruct=None)
        tag = f"w{w_bit}a{a_bit}qa{int(qa)}"
        names = []
        for name, m in net.named_modules():
            if type(m).__name__ in ("WxAxLinear", "WxAxConv2d"):
                names.append(f"{name}|{type(m).__name__}|{m.output_quant_name}")
        out[f"{tag}_layers"] = np.array(sorted(names))
        for k, v in orig.items():
            out[f"{tag}_orig|{k}"] = v
        for k, v in net.state_dict().items():
            out[f"{tag}_quant|{k}"] = v.numpy()
        x = rnd(rng, (2, 4, 8, 8), 1.0, outliers=3)
        out[f"{tag}_x"] = x
        with torch.no_grad():
            h = net.conv_in(t16(x))
            out[f"{tag}_conv_in_y"] = h.numpy()
            t = rnd(rng, (2, 5, 64), 1.0, outliers=2)
            out[f"{tag}_tok"] = t
            out[f"{tag}_add_k_proj_y"] = net.blk.add_k_proj(t16(t)).numpy()


def main():
    ref = _refload.load_reference()
    for fname, fn in (("fake_quant_golden.npz", gen_fake_quant),
                      ("smooth_golden.npz", gen_smooth),
                      ("install_golden.npz", gen_install)):
        out = {}
        with torch.no_grad():  # the reference runs under @torch.no_grad() (base.py:214)
            fn(ref, out)
        path = os.path.join(HERE, fname)
        np.savez_compressed(path, **out)
        print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path) / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
