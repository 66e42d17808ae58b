# k_colmax_nhwc geometry sweep under rocprofv3 (kernel durations, one process per setting)
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for cfg in "512 16" "512 64" "128 64" "32 64" "8 256"; do
set -- $cfg
timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cm_$1_$2 -o run -- python3 $R/scripts/colmax_sweep.py $1 $2 > /dev/null 2>&1
done
