set -o pipefail
bash scripts/gpu_step.sh w4_tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "int4_lds or weight_codes or linear_formats or skinny or geglu_epilogue or gemm_variants or attention" || exit 99
bash scripts/gpu_step.sh w4_shapes 300 python -u scripts/shape_bench.py --w4 --mscale 2 || exit 99
