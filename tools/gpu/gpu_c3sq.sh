#!/bin/bash
# SQ instruction counters of the scan kernels on C3 and C2 (one pass each)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3sq
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES"
for c in c3 c2; do
  timeout -s KILL 200 rocprofv3 --pmc $S2 --kernel-trace --output-format csv -d gpurun_out/c3sq/$c -o run -- python3 tools/scan_once.py $c 2 > gpurun_out/c3sq/$c.log 2>&1 || exit $?
done
echo done
