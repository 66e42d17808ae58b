# full GPU check (part 2): re-tuned table, determinism, the secondary bench lines, rocprof profiles
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh o_tune 600 python -u scripts/tune_table.py --out gpurun_out/gemm_table.json || exit 99
export QD_GEMM_TABLE=$PWD/gpurun_out/gemm_table.json
cp gpurun_out/gemm_table.json quantization---diffusion-models_amd/gemm_table.json
bash scripts/gpu_step.sh o_determinism 600 python -u -m pytest tests/test_gpu_determinism.py -q --timeout 900 -rf || exit 99
bash scripts/gpu_step.sh o_bench_int8 300 python -u bench.py --mode w8a8-sq-int8 --no-cpu-baseline --no-e2e || exit 99
bash scripts/gpu_step.sh o_bench_sdxl 300 python -u bench.py --model sdxl --steps 2 --no-cpu-baseline || exit 99
bash scripts/gpu_step.sh o_bench_sd35 300 python -u bench.py --model sd35 --denoise-steps 10 --steps 2 --no-cpu-baseline || exit 99
