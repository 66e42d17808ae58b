"""Diagnose test_groupnorm_fq_in_matches_finalize_then_norm[0-True-256]: repeat the case, report
where the fused (fq_in) GroupNorm and finalize -> GroupNorm differ and whether either side
changes between repeats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import qdiff_boot  # noqa: E402,F401
from qdiff import kernels as k  # noqa: E402


def case(bits, with_cadd, hw, dev="cuda:0"):
    g = torch.Generator().manual_seed(bits * 3 + with_cadd + hw)
    n, c = 2, 640
    y = (torch.randn(n, hw, c, generator=g) * 1.5).half().to(dev)
    amax = y.float().abs().amax(dim=1).reshape(-1).contiguous() if bits else None
    big = (torch.randn(n, 2 * c, generator=g) * 0.3).half().to(dev)
    cadd = big[:, 800: 800 + c] if with_cadd else None
    gam = (1 + 0.1 * torch.randn(c, generator=g)).half()
    bet = (0.1 * torch.randn(c, generator=g)).half()
    gam[::37] = 0.01
    bet[::37] = -0.5
    gam, bet = gam.to(dev), bet.to(dev)
    outs = []
    for _ in range(4):
        fin = k.fq_finalize(y, amax, bits, chan_add=cadd)
        ref = k.groupnorm_nhwc(fin, 32, 1e-5, gam, bet, silu=True, q_bits=8)
        got = k.groupnorm_nhwc(y, 32, 1e-5, gam, bet, silu=True, q_bits=8, fq_in=(amax, bits, cadd))
        torch.cuda.synchronize()
        outs.append((fin.clone(), ref.clone(), got.clone()))
    tf = (y.float() + cadd.float()).half() if cadd is not None else y
    print(f"case bits={bits} cadd={with_cadd} hw={hw}: fin == torch add: {torch.equal(outs[0][0], tf)}")
    for i, (fin, ref, got) in enumerate(outs):
        d = (got != ref)
        print(f"  rep {i}: fin stable {torch.equal(fin, outs[0][0])} ref stable {torch.equal(ref, outs[0][1])} "
              f"got stable {torch.equal(got, outs[0][2])} mismatches {int(d.sum())}")
        if d.any():
            idx = d.nonzero()[:8].tolist()
            for nn, r, ch in idx:
                print(f"    [{nn},{r},{ch}] got {got[nn, r, ch].item()} ref {ref[nn, r, ch].item()}")
            chs = sorted(set(d.nonzero()[:, 2].tolist()))
            print(f"    channels {chs[:20]} ({len(chs)})")


if __name__ == "__main__":
    for a in ((8, True, 256), (0, True, 256), (4, True, 256), (0, False, 256), (0, True, 64)):
        case(*a)
