set -o pipefail
bash scripts/gpu_step.sh u_tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -rf -k "tile_pingpong or (gemm_variants and (116 or 117 or 150 or 151 or 152))" || exit 99
bash scripts/gpu_step.sh u_lin_f16 400 python -u scripts/shape_bench.py --only linear --iters 10 || exit 99
bash scripts/gpu_step.sh u_lin_i8 400 python -u scripts/shape_bench.py --int8 --only linear --iters 10 || exit 99
