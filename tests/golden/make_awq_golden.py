"""Golden vectors of the reference's int4 AWQ packing utilities (TEST INFRASTRUCTURE; run ONCE in
the build container, needs /root/reference):

    python tests/golden/make_awq_golden.py

utils/quant_utils.py (pack / unpack / apply_order / dequantize, :14-67, :70-113) and
utils/packing_utils.py (unpack_awq / reverse_awq_order / dequantize_gemm, :8-40, :80-102) are
loaded in place (both import only torch) and fed seeded 4-bit matrices; the inputs and outputs are
written to tests/golden/awq_pack_golden.npz.  No reference source enters the repository.
"""
import importlib.util
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    qu = _load("ref_quant_utils", os.path.join(REF, "utils", "quant_utils.py"))
    pu = _load("ref_packing_utils", os.path.join(REF, "utils", "packing_utils.py"))
    rng = np.random.default_rng(44)
    out = {}
    K, N, g = 256, 64, 128
    iw = rng.integers(0, 16, (K, N)).astype(np.int8)          # AWQ layout: [in_features, out_features]
    iz = rng.integers(0, 16, (K // g, N)).astype(np.int8)
    sc = (rng.random((K // g, N)) * 0.05 + 0.001).astype(np.float16)
    t = lambda a: torch.from_numpy(a)
    ordered = qu.apply_order(t(iw).clone(), direction="column", order=qu.AWQ_PACK_ORDER)
    qweight = qu.pack(ordered, direction="column")
    qzeros = qu.pack(qu.apply_order(t(iz).clone(), direction="column", order=qu.AWQ_PACK_ORDER), direction="column")
    out["iweight"], out["izeros"], out["scales"] = iw, iz, sc
    out["qweight"], out["qzeros"] = qweight.numpy(), qzeros.numpy()
    uw, uz = pu.unpack_awq(qweight, qzeros, 4)
    uw, uz = pu.reverse_awq_order(uw, uz, 4)
    out["unpacked_iweight"] = torch.bitwise_and(uw, 15).numpy()
    out["unpacked_izeros"] = torch.bitwise_and(uz, 15).numpy()
    out["dequantize_gemm"] = pu.dequantize_gemm(qweight, qzeros, t(sc), 4, g).to(torch.float16).numpy()
    ex_w, ex_z = qu.awq_to_exllama(qweight, qzeros)
    out["exllama_qweight"], out["exllama_qzeros"] = ex_w.numpy(), ex_z.numpy()
    path = os.path.join(HERE, "awq_pack_golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays")


if __name__ == "__main__":
    main()
