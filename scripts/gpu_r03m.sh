set -o pipefail
QD_NO_I8_AMAX_FUSE=1 bash scripts/gpu_step.sh ab_gn_int8 600 bash scripts/ab.sh 2 --mode w8a8-sq-int8 --no-e2e || exit 99
bash scripts/gpu_step.sh ab_gn_fq 600 bash scripts/ab.sh 2 --no-e2e || exit 99
