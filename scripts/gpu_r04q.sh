# block order weighed by operand bytes: same-box A/Bs of QD_NO_MFAST on SD3.5 (int4 weights), SD1.5 fake-quant, int8
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04q_ab_sd35 600 bash scripts/ab_env.sh QD_NO_MFAST=1 2 --model sd35 --denoise-steps 10 --steps 2 --no-e2e || exit 99
bash scripts/gpu_step.sh r04q_ab_int8 600 bash scripts/ab_env.sh QD_NO_MFAST=1 2 --mode w8a8-sq-int8 --no-e2e || exit 99
