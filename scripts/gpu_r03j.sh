set -o pipefail
bash scripts/gpu_step.sh split_tests 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm_variants" || exit 99
bash scripts/gpu_step.sh retune_all 600 python -u scripts/tune_table.py --out gpurun_out/gemm_table.json || exit 99
NEW_TABLE=$PWD/gpurun_out/gemm_table.json bash scripts/gpu_step.sh ab_split 600 bash scripts/ab_table.sh 2 || exit 99
