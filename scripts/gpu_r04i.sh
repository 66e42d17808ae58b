# streaming short-K tiles: parity tests, short-K sweep (all variants), attention + short-K PMC
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_step.sh r04i_tests 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_int8.py -x -q -k "streaming or linear_i8" --timeout 300 --timeout-method thread -rf || exit 99
grep -q " passed" gpurun_out/r04i_tests.log && ! grep -q "failed" gpurun_out/r04i_tests.log || exit 98
bash scripts/gpu_step.sh r04i_shortk 400 python -u scripts/shortk_i8.py || exit 99
bash scripts/gpu_step.sh r04i_pmc_shortk 300 bash scripts/pmc_shortk.sh || exit 99
bash scripts/gpu_step.sh r04i_pmc_attn 300 bash scripts/pmc_attn2.sh || exit 99
