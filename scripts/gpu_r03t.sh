set -o pipefail
bash scripts/gpu_step.sh t_lin_f16 400 python -u scripts/shape_bench.py --only linear --iters 10 || exit 99
bash scripts/gpu_step.sh t_lin_i8 400 python -u scripts/shape_bench.py --int8 --only linear --iters 10 || exit 99
