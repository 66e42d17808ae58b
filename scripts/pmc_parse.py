"""Reduce scripts/pmc_traffic.sh output (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes)
to profiles/<tag>_pmc_dominant.json: HBM bytes per launch of the dominant conv (fp16 halo and the
int8-MFMA mode's halo) per GEMM variant, with the MI355X_MICROARCH.md gfx950 corrections
(FETCH_SIZE x2: it reports half of the 16-B/lane streaming reads; WRITE_SIZE as is; KB = 1024 B).
usage: python scripts/pmc_parse.py gpurun_out/pmc_TAG OUT.json "f16:202 i8:142" """
import csv
import glob
import json
import os
import sys

d, out, variants = sys.argv[1], sys.argv[2], sys.argv[3].split()
# the step's forms (scripts/roof_kernel.py): int8 adds the GroupNorm slot moments (16 B per 64-row slot
# and column) to codes + weights + fp16 output
ALG = {"f16": 8 * 64 * 64 * 320 * 2 + 320 * 9 * 320 * 2 + 8 * 64 * 64 * 320 * 2,
       "i8": 8 * 64 * 64 * 320 * 1 + 320 * 9 * 320 * 1 + 8 * 64 * 64 * 320 * 2 + 8 * 64 * 64 // 64 * 320 * 16}


def per_launch(path, counter):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    tot, disp = {}, set()
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"]
            if "k_gemm" not in k and "k_conv_halo" not in k:
                continue
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
            disp.add((k, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
    if not tot:
        return None, None, 0
    k = max(tot, key=tot.get)
    n = len([1 for kk, _ in disp if kk == k])
    return k, tot[k] / n, n


res = {"shape": "conv3x3 320->320 @64x64 b8 (M=32768,N=320,K=2880)",
       "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE reports 1/2 of 16-B/lane "
                     "streaming reads); WRITE_SIZE as is; KB = 1024 B",
       "algorithmic_bytes_per_launch": ALG["f16"],
       "algorithmic_bytes_per_launch_i8": ALG["i8"],
       "command": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) -- python3 scripts/roof_kernel.py "
                  "10 <variant> [--i8]",
       "forms": {"f16": "bias + output-fake-quant amax epilogue, pre-zeroed amax (the step's form)",
                 "i8": "bias + time-embedding add + GroupNorm slot statistics (the step's resnet conv1)"},
       "by_variant": {}}
for mv in variants:
    mode, v = mv.split(":")
    kf, fetch, nf = per_launch(os.path.join(d, f"{mode}_FETCH_SIZE_{v}"), "FETCH_SIZE")
    kw, write, nw = per_launch(os.path.join(d, f"{mode}_WRITE_SIZE_{v}"), "WRITE_SIZE")
    if fetch is None or write is None:
        continue
    hbm = int(round((2 * fetch + write) * 1024))
    rec = {"FETCH_SIZE_KB_per_launch": fetch, "WRITE_SIZE_KB_per_launch": write, "launches": nf,
           "kernel_name": kf, "hbm_bytes_per_launch": hbm,
           "read_bytes_per_launch": int(round(2 * fetch * 1024)), "write_bytes_per_launch": int(round(write * 1024)),
           "traffic_over_algorithmic": round(hbm / ALG[mode], 3)}
    res["by_variant"][v if mode == "f16" else f"i8:{v}"] = rec
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
