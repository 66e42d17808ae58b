"""Where the int8-MFMA mode's error comes from (CPU, build container): one full-size SD1.5 W8A8
eval at CFG batch 2 through the fp32 oracle with the int8 mode on every eligible layer, on the
convs only, on the linears only, against the unquantized fp16 UNet (and the reference's fake-quant
W8A8 for scale).  usage: python scripts/i8_error_split.py   (output: profiles/r03_i8_error_split.log)"""
import sys, time, numpy as np, torch
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import qdiff_boot
from oracle import config_cases as CC, int8_ref as I8, fake_quant_np as FQ
from oracle.unet_ref import RefUNet
from qdiff.unet import SD15, UNet2DConditionModel
torch.set_num_threads(8)
net = UNet2DConditionModel(SD15).half().init_synthetic(0)
sd = {k: v.detach() for k, v in net.state_dict().items()}
del net
cfg = CC.cfgdict(SD15)
g = torch.Generator().manual_seed(42)
x = torch.randn(2, 4, 64, 64, generator=g).half()
ctx = torch.randn(2, 77, 768, generator=g).half()
QC8 = dict(w_bit=8, a_bit=8, q_group_size=128, quantize_act=True)
t0 = time.time()
r16 = RefUNet(cfg, sd, None, variant="fp32").forward(x, 981, ctx).float(); print("fp16", time.time()-t0, flush=True)
rfq = RefUNet(cfg, sd, QC8, variant="fp32").forward(x, 981, ctx).float(); print("fq", time.time()-t0, flush=True)
ri8 = RefUNet(cfg, sd, QC8, variant="fp32", int8=True).forward(x, 981, ctx).float(); print("i8", time.time()-t0, flush=True)
# variant: int8 convs only (linears keep the fake-quant A16 path)
class ConvOnly(RefUNet):
    def _int8_weights(self, sd):
        out = super()._int8_weights(sd)
        for n in [k for k, v in self.i8.items() if v[0] == "linear"]:
            del self.i8[n]; out[n + ".weight"] = sd[n + ".weight"]
        return out
rc = ConvOnly(cfg, sd, QC8, variant="fp32", int8=True).forward(x, 981, ctx).float(); print("i8 conv only", time.time()-t0, flush=True)
class LinOnly(RefUNet):
    def _int8_weights(self, sd):
        out = super()._int8_weights(sd)
        for n in [k for k, v in self.i8.items() if v[0] == "conv"]:
            del self.i8[n]; out[n + ".weight"] = sd[n + ".weight"]
        return out
rl = LinOnly(cfg, sd, QC8, variant="fp32", int8=True).forward(x, 981, ctx).float(); print("i8 lin only", time.time()-t0, flush=True)
sc = r16.abs().max().item()
rel = lambda a, b: ((a - b).abs().max().item() / sc, (a - b).abs().mean().item() / sc)
print("fake-quant vs fp16", rel(rfq, r16))
print("int8 all vs fp16", rel(ri8, r16))
print("int8 conv only (linears fake-quant A16) vs fp16", rel(rc, r16))
print("int8 linears only (convs fake-quant) vs fp16", rel(rl, r16))
