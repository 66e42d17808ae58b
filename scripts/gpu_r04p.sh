# block order weighed by operand bytes: same-box A/Bs of QD_NO_MFAST on SD3.5 (int4 weights), SD1.5 fake-quant, int8
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04p_ab_sd35 600 bash scripts/ab_env.sh QD_NO_MFAST=1 2 --model sd35 --denoise-steps 10 --steps 2 --no-e2e || exit 99
bash scripts/gpu_step.sh r04p_ab_fq 500 bash scripts/ab_env.sh QD_NO_MFAST=1 2 --no-e2e || exit 99
bash scripts/gpu_step.sh r04p_ab_sdxl 500 bash scripts/ab_env.sh QD_NO_MFAST=1 1 --model sdxl --steps 2 --no-e2e || exit 99
bash scripts/gpu_step.sh r04p_qrows_def 200 python -u scripts/i8_bench.py || exit 99
bash scripts/gpu_step.sh r04p_qrows_r4 200 env QD_QROWS_R=4 python -u scripts/i8_bench.py || exit 99
bash scripts/gpu_step.sh r04p_qrows_r1 200 env QD_QROWS_R=1 python -u scripts/i8_bench.py || exit 99
