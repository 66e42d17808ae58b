"""Summarise a rocprofv3 rocpd database: per-kernel totals (optionally per UNet eval).
usage: python scripts/prof_summary.py gpurun_out/prof_X/run_results.db [evals_kernel_substring]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                  "order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
marker = sys.argv[2] if len(sys.argv) > 2 else "k_cfg_ddim"
evals = sum(r[1] for r in rows if marker in r[0]) or 1
print(f"total {tot / 1e6:.2f} ms over {evals} evals ({marker}) -> {tot / 1e6 / evals:.3f} ms/eval")
print(f"{'ms/eval':>8} {'calls/eval':>10} {'avg us':>8}  kernel")
for name, n, s, a in rows[:45]:
    print(f"{s / 1e6 / evals:8.3f} {n / evals:10.2f} {a / 1e3:8.1f}  {name[:100]}")
