# int8 halo conv with 128-pixel tiles (2 blocks / CU, variants 145-147) + single-pass slot merge:
# tests, variant sweep, re-tune of the int8 keys, A/B of the tables, profile
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04e_tests 700 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 300 --timeout-method thread -rf || exit 99
bash scripts/gpu_step.sh r04e_sweep 300 python -u scripts/i8_bench.py --sweep || exit 99
bash scripts/gpu_step.sh r04e_tune 300 python -u scripts/tune_table.py --add --drop-epi 511 --models sd15 --out gpurun_out/gemm_table.json || exit 99
export QD_GEMM_TABLE=$PWD/gpurun_out/gemm_table.json
bash scripts/gpu_step.sh r04e_ab_table 600 bash scripts/ab_env.sh QD_GEMM_TABLE=$PWD/quantization---diffusion-models_amd/gemm_table.json 2 --mode w8a8-sq-int8 --no-e2e || exit 99
bash scripts/prof_bench.sh r04e_int8 400 --mode w8a8-sq-int8 --no-e2e || exit 99
