set -o pipefail
bash scripts/gpu_step.sh retune_i4 500 python -u scripts/tune_table.py --retune-i4 --out gpurun_out/gemm_table.json || exit 99
export QD_GEMM_TABLE=$PWD/gpurun_out/gemm_table.json
bash scripts/gpu_step.sh sd35_codes 300 python -u bench.py --model sd35 --denoise-steps 10 --steps 2 --no-cpu-baseline || exit 99
QD_W4_OPERAND=tuned bash scripts/gpu_step.sh sd35_tuned 300 python -u bench.py --model sd35 --denoise-steps 10 --steps 2 --no-cpu-baseline || exit 99
bash scripts/gpu_step.sh sd15_bench 300 python -u bench.py --no-cpu-baseline || exit 99
bash scripts/gpu_step.sh gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf || exit 99
