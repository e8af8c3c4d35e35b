#!/bin/bash
# stall/activity counters of the scan kernels: tools/gpu/gpu_pmc2.sh OUT CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/$1; shift
mkdir -p $D
export TMPDIR=/tmp
S3="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
for cfg in "$@"; do
  T="tools/scan_once.py $cfg 2"; [ $cfg = small ] && T="tools/small_once.py"
  timeout -s KILL 200 rocprofv3 --pmc $S3 --kernel-trace --output-format csv -d $D/${cfg}_p3 -o run -- python3 $T > $D/${cfg}_p3.log 2>&1 || exit $?
done
python3 tools/pmc_agg.py $D "$@" | grep -A10 "k_scan"
