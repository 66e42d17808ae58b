"""Debug: where does the HIP WxAxLinear differ from the reference's golden F.linear output?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import qdiff_boot  # noqa
from qdiff.fake_quant import WxAxLinear
from qdiff import kernels as K
g = np.load("tests/golden/fake_quant_golden.npz")
dev = torch.device("cuda:0")
for key in ["lin_w4_qo0", "lin_w8_qo0"]:
    w, b = torch.from_numpy(g[key + "_w"]), torch.from_numpy(g[key + "_b"])
    lin = torch.nn.Linear(320, 640).half().to(dev)
    with torch.no_grad():
        lin.weight.copy_(w); lin.bias.copy_(b)
    m = WxAxLinear.from_float(lin, weight_quant="group", n_bits_W=4 if "w4" in key else 8, group_size_W=128)
    x = torch.from_numpy(g[key + "_x"])
    y = torch.from_numpy(g[key + "_y"]).float()
    for force in [None, 0, 1, 2, 3]:
        K.force_gemm(force)
        got = m(x.to(dev)).cpu().float()
        K.force_gemm(None)
        d = (got - y).abs()
        i = d.argmax()
        r, c = divmod(i.item(), 640)
        f64 = (x.double().view(-1, 320)[r] @ m.weight.cpu().double()[c] + b.double()[c]).item()
        print(key, "force", force, "max", d.max().item(), "n>0", (d > 0).sum().item(), "at", (r, c), "ref", y.view(-1, 640)[r, c].item(),
              "got", got.view(-1, 640)[r, c].item(), "f64", f64, "choices", [v for k_, v in K.gemm_choices().items() if k_[1] == 154])
    got = m(x.to(dev)).cpu().float()
    u = torch.pow(2.0, torch.floor(torch.log2(torch.maximum(got.abs(), y.abs()).clamp(min=6.1e-5))) - 10)
    bad = ((got - y).abs() > 2 * u).nonzero()
    for idx in bad[:10]:
        idx = tuple(idx.tolist())
        r = idx[0] * 77 + idx[1]
        f64 = (x.double().view(-1, 320)[r] @ m.weight.cpu().double()[idx[2]] + b.double()[idx[2]]).item()
        print("  bad", idx, "ref", y[idx].item(), "got", got[idx].item(), "f64", f64, "2u", 2 * u[idx].item())
