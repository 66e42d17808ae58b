set -o pipefail
bash scripts/gpu_step.sh epi_tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "int4_lds or linear_formats or gemm_variants or post_residual or conv" || exit 99
bash scripts/gpu_step.sh ab_resid 600 bash scripts/ab.sh 2 || exit 99
bash scripts/gpu_step.sh retune_i4 500 python -u scripts/tune_table.py --retune-i4 --out gpurun_out/gemm_table.json || exit 99
export QD_GEMM_TABLE=$PWD/gpurun_out/gemm_table.json
bash scripts/gpu_step.sh sd35_tuned 300 python -u bench.py --model sd35 --denoise-steps 10 --steps 2 --no-cpu-baseline || exit 99
QD_W4_OPERAND=codes bash scripts/gpu_step.sh sd35_codes 300 python -u bench.py --model sd35 --denoise-steps 10 --steps 2 --no-cpu-baseline || exit 99
bash scripts/gpu_step.sh c3_tuned 400 python -u bench.py --mode w4a16 --batch 8 --no-cpu-baseline --no-e2e --steps 2 || exit 99
