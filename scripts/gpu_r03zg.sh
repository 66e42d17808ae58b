set -o pipefail
bash scripts/prof_bench.sh r03zg 400 || exit 99
bash scripts/prof_bench.sh r03zg_int8 400 --mode w8a8-sq-int8 --no-e2e || exit 99
