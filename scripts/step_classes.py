"""Group one denoising step's kernels (rocprofv3 kernel trace) into classes: share of the step
and launch counts, as the r01 verdict's table.
usage: python scripts/step_classes.py gpurun_out/prof_X/run_kernel_trace.csv [marker] [which=-2]"""
import csv
import sys

CLASSES = [("GEMM/conv", ("k_gemm", "k_conv_halo", "k_gemv", "k_geglu_i8q")), ("split-K reduce", ("k_splitk",)),
           ("attention", ("k_attn",)), ("GroupNorm", ("k_gn_",)), ("LayerNorm", ("k_layernorm", "k_ln_rows", "k_fq_layernorm")),
           ("finalize", ("k_finalize",)), ("colmax + apply", ("k_colmax", "k_apply", "k_act_")),
           ("int8 act quant", ("k_quant_rows_i8", "k_quant_rows_g", "k_sample_", "k_cat_apply_i8")), ("scheduler / embed", ("k_cfg", "k_timestep")),
           ("elementwise", ("k_silu", "k_add", "k_concat", "k_geglu", "k_zero", "k_nchw", "k_nhwc"))]

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_cfg_ddim"
which = int(sys.argv[3]) if len(sys.argv) > 3 else -2
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(path)))
marks = [i for i, e in enumerate(ev) if marker in e[2]]
a, b = marks[which - 1] + 1, marks[which] + 1
agg = {}
tot = 0
for s, e, n in ev[a:b]:
    cls = next((c for c, keys in CLASSES if any(k in n for k in keys)), "other")
    r = agg.setdefault(cls, [0, 0])
    r[0] += e - s
    r[1] += 1
    tot += e - s
print(f"step kernels {tot / 1e6:.3f} ms, launches {b - a}")
print(f"{'class':<20} {'ms':>8} {'share':>7} {'launches':>9}")
for cls, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{cls:<20} {t / 1e6:8.3f} {100 * t / tot:6.1f}% {n:9d}")
