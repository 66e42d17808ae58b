# attention PMC (16x16x32 vs 32x32x16 at d = 40), short-K linear timing sweep + PMC
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04h_pmc_attn 400 bash scripts/pmc_attn2.sh || exit 99
bash scripts/gpu_step.sh r04h_shortk 400 python -u scripts/shortk_i8.py || exit 99
bash scripts/gpu_step.sh r04h_pmc_shortk 400 bash scripts/pmc_shortk.sh || exit 99
