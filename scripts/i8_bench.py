"""int8 vs fp16 GEMM/conv timing on the SD1.5 CFG-batch-8 shapes (HIP events; each path tuned).
usage: python scripts/i8_bench.py [--iters 20]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as K  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--sweep", action="store_true", help="also time every forced int8 conv variant")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    # (n, h, w, cin, cout, k, stride, count per eval)
    convs = [(8, 64, 64, 320, 320, 3, 1, 7), (8, 32, 32, 640, 640, 3, 1, 6), (8, 16, 16, 1280, 1280, 3, 1, 7),
             (8, 8, 8, 1280, 1280, 3, 1, 8), (8, 64, 64, 640, 320, 3, 1, 2), (8, 32, 32, 1280, 640, 3, 1, 2),
             (8, 16, 16, 2560, 1280, 3, 1, 2), (8, 64, 64, 320, 320, 1, 1, 10)]
    print("conv (n,h,w,ci,co,k): f16 us | i8 us | speedup | i8 TOPS | choice")
    for (n, h, w, ci, co, k, s, cnt) in convs:
        x = torch.randn(n, h, w, ci, generator=g).half().to(dev)
        wt = (torch.randn(co, k, k, ci, generator=g) / (k * k * ci) ** 0.5).half().to(dev)
        b = torch.zeros(co, dtype=torch.float16, device=dev)
        tf = timeit(lambda: K.conv2d_nhwc(x, wt, ci, s, k // 2, bias=b), a.iters)
        xq, sa = K.quant_samples_i8(x)
        wq, sw16, _ = K.weight_quant(wt.view(co, -1).contiguous(), k * k * ci, 8, want_dq=False)
        wq = wq.view(co, k, k, ci)
        sw = sw16.float().view(-1).contiguous()
        ti = timeit(lambda: K.conv2d_i8(xq, sa, wq, sw, ci, s, k // 2, bias=b), a.iters)
        flops = 2.0 * n * h * w * co * k * k * ci / (s * s)
        ch = [v for kk, v in K.gemm_choices().items() if kk[0] == "conv_i8" and kk[1:6] == (n, h, w, ci, co)]
        print(f"({n},{h},{w},{ci},{co},{k}) x{cnt}: {tf:8.1f} | {ti:8.1f} | {tf / ti:5.2f} | {flops / ti / 1e6:7.1f} | {ch}")
        if a.sweep:
            ref = K.conv2d_i8(xq, sa, wq, sw, ci, s, k // 2, bias=b)
            row = []
            for v in K.I8_VARIANTS + K.I8_HALO_VARIANTS:
                K.force_gemm(v)
                try:
                    tv = timeit(lambda: K.conv2d_i8(xq, sa, wq, sw, ci, s, k // 2, bias=b), a.iters)
                    same = torch.equal(K.conv2d_i8(xq, sa, wq, sw, ci, s, k // 2, bias=b), ref)
                    row.append(f"{v}:{tv:.1f}{'' if same else '(DIFF)'}")
                except RuntimeError as e:
                    row.append(f"{v}:err")
                finally:
                    K.force_gemm(None)
            print("    sweep us:", " ".join(row), flush=True)
    lins = [(32768, 320, 320), (32768, 2560, 320), (32768, 320, 1280), (8192, 640, 640), (8192, 5120, 640),
            (2048, 1280, 1280), (2048, 10240, 1280), (8192, 640, 2560), (616, 320, 768)]
    print("linear (M,N,K): f16 us | i8 us | speedup | i8 TOPS")
    for (m, nn, kk) in lins:
        x = torch.randn(m, kk, generator=g).half().to(dev)
        wt = (torch.randn(nn, kk, generator=g) / kk ** 0.5).half().to(dev)
        tf = timeit(lambda: K.linear(x, wt), a.iters)
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(wt, kk, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()
        ti = timeit(lambda: K.linear_i8(xq, sa, wq, sw), a.iters)
        tq = timeit(lambda: K.quant_rows_i8(x), a.iters)
        flops = 2.0 * m * nn * kk
        print(f"({m},{nn},{kk}): {tf:8.1f} | {ti:8.1f} | {tf / ti:5.2f} | {flops / ti / 1e6:7.1f} | row-quant {tq:6.1f} us")


if __name__ == "__main__":
    main()
