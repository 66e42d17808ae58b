#!/bin/bash
# One GPU call: gpu tests, the default bench line, and a rocprofv3 kernel-trace of one bench step.
# usage: scripts/round_gpu.sh TAG   (results under gpurun_out/)
set -o pipefail
TAG=${1:-r}
cd "$(dirname "$0")/.."
bash scripts/gpu_step.sh tests_$TAG 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 99
bash scripts/gpu_step.sh bench_$TAG 400 python -u bench.py || exit 99
bash scripts/prof_bench.sh $TAG 400 || exit 99
