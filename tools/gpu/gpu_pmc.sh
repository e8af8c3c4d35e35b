#!/bin/bash
# SQ instruction counts of the scan kernels: tools/gpu/gpu_pmc.sh OUT CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/$1; shift
mkdir -p $D
export TMPDIR=/tmp
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES"
for cfg in "$@"; do
  T="tools/scan_once.py $cfg 2"; [ $cfg = small ] && T="tools/small_once.py"
  timeout -s KILL 200 rocprofv3 --pmc $S2 --kernel-trace --output-format csv -d $D/${cfg}_p1 -o run -- python3 $T > $D/${cfg}_p1.log 2>&1 || exit $?
done
python3 tools/pmc_agg.py $D "$@" | grep -A10 "k_scan\|k_emit"
