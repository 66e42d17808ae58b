set -o pipefail
bash scripts/gpu_step.sh attn_tests 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_encdec.py -x -q --timeout 120 --timeout-method thread -k "attention or clip or vae" || exit 99
bash scripts/gpu_step.sh attn_ab 200 bash -c 'for r in 1 2; do for l in prev new; do if [ $l = prev ]; then export QD_LIB_PATH=$PWD/scripts/ab/libqdiff_prev.so; else unset QD_LIB_PATH; fi; echo "== $l"; python -u scripts/attn_bench.py; done; done' || exit 99
bash scripts/gpu_step.sh ab_attn_bench 600 bash scripts/ab.sh 2 || exit 99
