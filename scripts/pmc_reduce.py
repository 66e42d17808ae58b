"""Per-dispatch averages of every PMC counter of the dominant k_gemm / k_conv kernel in each pass
directory of a scripts/pmc_*.sh run.  usage: python scripts/pmc_reduce.py gpurun_out/pmc_TAG"""
import csv
import glob
import os
import sys

root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*_*"))):
    if not os.path.isdir(d):
        continue
    vals, disp = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_gemm" not in k and "k_conv" not in k:
                continue
            key = (k, r["Counter_Name"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
            disp.setdefault(key, set()).add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    kern = {}
    for (k, c), v in vals.items():
        kern.setdefault(k, {})[c] = v / max(len(disp[(k, c)]), 1)
    for k, cs in kern.items():
        print(os.path.basename(d), k[:60])
        for c in sorted(cs):
            print(f"    {c:32s} {cs[c]:16.4g}")
