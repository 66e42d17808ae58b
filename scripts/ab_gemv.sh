# skinny-M GEMV A/B: GPU suite, then each bench line with the GEMV (default) and without (QD_NO_GEMV=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gv_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --model sd35 --denoise-steps 10 --steps 2 > gpurun_out/gv_sd35_on.log 2>&1 || exit 1
QD_NO_GEMV=1 timeout -k 10 300 python3 bench.py --model sd35 --denoise-steps 10 --steps 2 > gpurun_out/gv_sd35_off.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/gv_sd15_on.log 2>&1 || exit 1
QD_NO_GEMV=1 timeout -k 10 300 python3 bench.py > gpurun_out/gv_sd15_off.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_gv -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model sd35 --denoise-steps 4 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/gv_prof.log 2>&1
