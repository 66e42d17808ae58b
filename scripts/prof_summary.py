"""Summarise a rocprofv3 kernel trace (csv or rocpd db): per-kernel time per UNet eval over the
LAST `evals` UNet evaluations of the run (default 50 = the timed generate of
`bench.py --steps 1`), so warm-up, calibration and GEMM-tuning launches are excluded.
usage: python scripts/prof_summary.py gpurun_out/prof_X/run_kernel_trace.csv [evals] [marker]"""
import sys

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 50
marker = sys.argv[3] if len(sys.argv) > 3 else "k_cfg_ddim"
if path.endswith(".csv"):
    import csv
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path))]
else:
    import sqlite3
    db = sqlite3.connect(path)
    ev = db.execute("select start, end, name from kernels").fetchall()
ev.sort()
marks = [i for i, e in enumerate(ev) if marker in e[2]]
if len(marks) > last:
    ev = ev[marks[-last - 1] + 1:]
evals = sum(1 for e in ev if marker in e[2]) or 1
agg = {}
for s, e, n in ev:
    a = agg.setdefault(n, [0, 0])
    a[0] += 1
    a[1] += e - s
rows = sorted(((k, n, t, t / n) for k, (n, t) in agg.items()), key=lambda r: -r[2])
tot = sum(r[2] for r in rows)
span = (ev[-1][1] - ev[0][0]) if ev else 0
print(f"last {evals} evals: kernel time {tot / 1e6 / evals:.3f} ms/eval, wall span {span / 1e6 / evals:.3f} ms/eval")
print(f"{'ms/eval':>8} {'calls/eval':>10} {'avg us':>8}  kernel")
for name, n, s, a in rows[:45]:
    print(f"{s / 1e6 / evals:8.3f} {n / evals:10.2f} {a / 1e3:8.1f}  {name[:100]}")
