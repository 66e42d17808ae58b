"""One denoising step's kernel sequence from a rocprofv3 kernel trace: duration of every launch
and the idle gap before it (graph replay), in launch order.
usage: python scripts/eval_sequence.py gpurun_out/prof_X/run_kernel_trace.csv [marker] [which=-2]"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_cfg_ddim"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
marks = [i for i, e in enumerate(ev) if marker in e[2]]
a, b = marks[which - 1] + 1, marks[which] + 1
prev_end = ev[a - 1][1]
tot_k = tot_g = 0
for s, e, n in ev[a:b]:
    gap = s - prev_end
    tot_k += e - s
    tot_g += max(gap, 0)
    print(f"{(e - s) / 1e3:8.1f} us  gap {gap / 1e3:6.1f}  {n[:90]}")
    prev_end = e
print(f"kernels {tot_k / 1e6:.3f} ms, gaps {tot_g / 1e6:.3f} ms, launches {b - a}")
