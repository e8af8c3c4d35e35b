#!/bin/bash
# SQ counter passes of the final build for next-round planning: k_scan on C2
# and C3, the merge kernels on C4 (one rocprofv3 --pmc run per set)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcr3
export TMPDIR=/tmp
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_IFETCH"
for cfg in c2 c3; do
  i=0
  for s in "$S1" "$S2"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $s --kernel-trace --output-format csv -d gpurun_out/pmcr3/${cfg}_p$i -o run -- python3 tools/scan_once.py $cfg 2 > gpurun_out/pmcr3/${cfg}_p$i.log 2>&1 || exit $?
  done
done
i=0
for s in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $s --kernel-trace --output-format csv -d gpurun_out/pmcr3/c4_p$i -o run -- python3 bench.py --config c4 --steps 1 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/pmcr3/c4_p$i.log 2>&1 || exit $?
done
exit 0
