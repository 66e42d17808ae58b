"""Same-process A/B of the two GEMM epilogue forms (qd_gemm_epi_lds 0 = direct fragment stores,
1 = LDS C tile) on the SD1.5 shapes they serve: the tuned kernel of each shape, interleaved rounds.
usage: python scripts/epi_ab.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import _lib  # noqa: E402
from qdiff import kernels as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    cases = []
    for (m, n, k) in ((32768, 2560, 320), (8192, 5120, 640), (2048, 10240, 1280)):  # GEGLU projections
        x = torch.randn(m, k, generator=g).half().to(dev)
        w = (torch.randn(n, k, generator=g) / k ** 0.5).half().to(dev)
        b = torch.randn(n, generator=g).half().to(dev)
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(w, k, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()
        cases.append((f"f16 geglu M{m} N{n} K{k}", lambda x=x, w=w, b=b: K.linear(x, w, "f16", bias=b, geglu=True)))
        cases.append((f"i8 geglu M{m} N{n} K{k}", lambda xq=xq, sa=sa, wq=wq, sw=sw, b=b:
                      K.linear_i8(xq, sa, wq, sw, bias=b, geglu=True)))
    for (m, c, kk) in ((32768, 320, 320), (8192, 640, 640), (32768, 320, 1280), (8192, 640, 2560), (32768, 960, 320)):
        x = torch.randn(m, kk, generator=g).half().to(dev)
        w = (torch.randn(c, kk, generator=g) / kk ** 0.5).half().to(dev)
        b = torch.randn(c, generator=g).half().to(dev)
        r = torch.randn(m, c, generator=g).half().to(dev)
        xq, sa = K.quant_rows_i8(x)
        wq, sw16, _ = K.weight_quant(w, kk, 8, want_dq=False)
        sw = sw16.float().view(-1).contiguous()
        cases.append((f"f16 lin+res M{m} N{c} K{kk}", lambda x=x, w=w, b=b, r=r: K.linear(x, w, "f16", bias=b, residual=r)))
        cases.append((f"i8 lin+res M{m} N{c} K{kk}", lambda xq=xq, sa=sa, wq=wq, sw=sw, b=b, r=r:
                      K.linear_i8(xq, sa, wq, sw, bias=b, residual=r)))
    for (n, hw, ci, co) in ((8, 64, 320, 320), (8, 32, 640, 640), (8, 16, 1280, 1280), (8, 64, 640, 320)):
        x = torch.randn(n, hw, hw, ci, generator=g).half().to(dev)
        w = (torch.randn(co, 3, 3, ci, generator=g) / (9 * ci) ** 0.5).half().to(dev)
        b = torch.randn(co, generator=g).half().to(dev)
        am = torch.zeros(n * co, dtype=torch.float32, device=dev)
        cases.append((f"f16 conv3x3+amax n{n} {hw}^2 {ci}->{co}", lambda x=x, w=w, b=b, am=am, ci=ci:
                      K.conv2d_nhwc(x, w, ci, 1, 1, bias=b, amax=am)))
    for name, fn in cases:
        fn()  # tune
        t = {0: [], 1: []}
        for _ in range(4):
            for mode in (0, 1):
                _lib.call("qd_gemm_epi_lds", mode)
                t[mode].append(timeit(fn))
        _lib.call("qd_gemm_epi_lds", 0)
        d, l = statistics.median(t[0]), statistics.median(t[1])
        print(f"{name:40s} direct {d:7.1f} us | lds {l:7.1f} us | {100 * (l - d) / l:+5.1f} %", flush=True)


if __name__ == "__main__":
    main()
