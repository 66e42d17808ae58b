#!/bin/bash
# A/B of one environment switch on ONE box: bench.py with VAR=VALUE ("prev") vs without ("new"), alternating.
# usage: bash scripts/ab_env.sh VAR=VALUE <rounds> [bench args...]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
KV=$1; shift
# the product reads four environment variables; the round-4/5 A/B switches
# (QD_NO_GN_PART, QD_NO_AMAX_POST, QD_NO_LN_EPI, QD_NO_FQ_REDUCE, QD_NO_GEMV, QD_NO_MFAST, QD_ATTN_CFG,
# QD_COLMAX_*) are retired: an A/B on them would compare two identical builds.  Kernel-choice A/Bs go
# through scripts/ab_flag.sh or the qd_*_force C-ABI knobs.
case "${KV%%=*}" in
  QD_GEMM_TABLE|QD_GEMM_TUNE|QD_LIB_PATH|QD_W4_OPERAND|QD_TUNE_COLD) ;;
  *) echo "[ab_env] ${KV%%=*} is not read by the product (live: QD_GEMM_TABLE QD_GEMM_TUNE QD_LIB_PATH QD_W4_OPERAND QD_TUNE_COLD)"; exit 2 ;;
esac
R=${1:-2}; shift
for i in $(seq 1 "$R"); do
  for side in prev new; do
    if [ "$side" = prev ]; then out=$(env "$KV" timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }
    else out=$(timeout -k 10 400 python -u "$ROOT/bench.py" --no-cpu-baseline "$@" 2>/dev/null | tail -1) || { echo "[ab] $side failed"; exit 1; }; fi
    echo "[ab] round $i $side: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], "int8_mode", (d.get("int8_mode") or {}).get("value"))')"
  done
done
