#!/bin/bash
# same-box A/B of qd_attn_force settings on the path's attention shapes, alternating rounds
# usage: bash scripts/attn_ab.sh "CFG_A CFG_B ..." [rounds]
CFGS=$1; R=${2:-2}
for i in $(seq 1 "$R"); do
  for c in $CFGS; do
    timeout -k 10 120 python3 scripts/attn_bench.py "$c" 2>&1 | grep -E "cfg=" | head -4 || exit 1
  done
done
