set -o pipefail
bash scripts/gpu_step.sh retune_i4 500 python -u scripts/tune_table.py --retune-i4 || exit 99
bash scripts/gpu_step.sh c3_tuned 400 python -u bench.py --mode w4a16 --batch 8 --no-cpu-baseline --no-e2e --steps 2 || exit 99
QD_W4_OPERAND=codes bash scripts/gpu_step.sh c3_codes 400 python -u bench.py --mode w4a16 --batch 8 --no-cpu-baseline --no-e2e --steps 2 || exit 99
