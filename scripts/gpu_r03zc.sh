set -o pipefail
bash scripts/gpu_step.sh zc_tests 400 python -u -m pytest tests/test_gpu_int8.py -x -q --timeout 120 --timeout-method thread -rf -k "bit_exact and not teacher" || exit 99
bash scripts/gpu_step.sh zc_tune 420 env QD_GEMM_TABLE=none python -u scripts/tune_table.py --out gpurun_out/gemm_table.json || exit 99
cp quantization---diffusion-models_amd/gemm_table.json gpurun_out/old_table.json && cp gpurun_out/gemm_table.json quantization---diffusion-models_amd/gemm_table.json || exit 99
bash scripts/gpu_step.sh zc_ab_int8 400 bash scripts/ab_env.sh QD_GEMM_TABLE=$PWD/gpurun_out/old_table.json 2 --mode w8a8-sq-int8 --no-e2e || exit 99
bash scripts/gpu_step.sh zc_ab_fq 400 bash scripts/ab_env.sh QD_GEMM_TABLE=$PWD/gpurun_out/old_table.json 2 --no-e2e || exit 99
