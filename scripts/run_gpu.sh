#!/bin/bash
# One parameterised GPU-box runner (replaces the per-round r05*.sh one-offs).  Every stage runs
# under its own time limit; the first fault / timeout / failure ends the call (no retries).
#
#   scripts/run_gpu.sh TAG STAGE [STAGE ...]
#
# stages (run in the order given; outputs under gpurun_out/TAG_*):
#   tests:<pytest args, ',' for spaces>   e.g. tests:tests/test_gpu_small_shapes.py (log: TAG_tests<n>.log)
#   suite          the full `-m gpu` suite (one process, thread timeouts)
#   smoke          __graft_entry__.smoke()
#   bench          the default bench line (fake-quant headline + int8_mode object), 20 steps
#   bench:<args>   bench.py with extra args (',' for spaces), e.g. bench:--model,sdxl
#   prof_fq        rocprofv3 step profile of the fake-quant mode (scripts/prof_bench.sh)
#   prof_int8      the same for the int8-MFMA mode
#   py:<script args, ',' for spaces>   a measurement script, 300 s limit (log: TAG_py<n>.log)
#   rprof:<script args>  the same under rocprofv3 --kernel-trace --stats (dir: TAG_rprof<n>/)
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
nt=0
np=0
for st in "$@"; do
  case "$st" in
    tests:*)
      args=${st#tests:}
      args=${args//,/ }
      nt=$((nt + 1))
      timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $args \
        > gpurun_out/${TAG}_tests${nt}.log 2>&1
      rc=$?; tail -5 gpurun_out/${TAG}_tests${nt}.log; [ $rc -eq 0 ] || exit 11 ;;
    suite)
      timeout -k 10 1000 python3 -u -m pytest tests -x -q --timeout 600 --timeout-method thread -m gpu \
        > gpurun_out/${TAG}_suite.log 2>&1
      rc=$?; tail -5 gpurun_out/${TAG}_suite.log; [ $rc -eq 0 ] || exit 12 ;;
    smoke)
      timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit 13 ;;
    bench)
      timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1
      rc=$?; tail -c 1200 gpurun_out/${TAG}_bench.log; [ $rc -eq 0 ] || exit 14 ;;
    bench:*)
      args=${st#bench:}
      args=${args//,/ }
      name=$(echo "$args" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)
      timeout -k 10 500 python3 bench.py $args > gpurun_out/${TAG}_bench_${name}.log 2>&1
      rc=$?; tail -c 800 gpurun_out/${TAG}_bench_${name}.log; [ $rc -eq 0 ] || exit 15 ;;
    prof_fq)
      timeout -k 10 450 bash scripts/prof_bench.sh ${TAG}_fq 400 > gpurun_out/${TAG}_prof_fq.log 2>&1 || exit 16
      head -14 gpurun_out/prof_${TAG}_fq/step_classes.txt ;;
    prof_int8)
      timeout -k 10 450 bash scripts/prof_bench.sh ${TAG}_int8 400 --mode w8a8-sq-int8 \
        > gpurun_out/${TAG}_prof_int8.log 2>&1 || exit 17
      head -14 gpurun_out/prof_${TAG}_int8/step_classes.txt ;;
    py:*)
      args=${st#py:}
      args=${args//,/ }
      np=$((np + 1))
      timeout -k 10 300 python3 -u $args > gpurun_out/${TAG}_py${np}.log 2>&1
      rc=$?; tail -5 gpurun_out/${TAG}_py${np}.log; [ $rc -eq 0 ] || exit 18 ;;
    rprof:*)
      args=${st#rprof:}
      args=${args//,/ }
      np=$((np + 1))
      od=$PWD/gpurun_out/${TAG}_rprof${np}
      mkdir -p "$od"
      (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$od" -o run \
        -- python3 -u $OLDPWD/$args) > "$od/run.log" 2>&1
      rc=$?; find "$od" -name "*kernel_trace.csv" -size +8M -delete
      tail -3 "$od/run.log"; [ $rc -eq 0 ] || exit 19 ;;
    *)
      echo "unknown stage $st"; exit 2 ;;
  esac
done
