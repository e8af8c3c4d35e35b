#!/bin/bash
# round 4: full GPU suite, then SQ counters of k_scan / k_emit on C2 and a kernel-stats pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4b/pytest_gpu.log 2>&1
echo "pytest rc=$?"; tail -8 gpurun_out/r4b/pytest_gpu.log
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
S2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT"
i=0
for s in "$S1" "$S2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $s --kernel-trace --output-format csv -d gpurun_out/r4b/c2_p$i -o run -- python3 tools/scan_once.py c2 2 > gpurun_out/r4b/c2_p$i.log 2>&1 || exit $?
done
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b/c2_stats -o run -- python3 tools/scan_once.py c2 10 > gpurun_out/r4b/c2_stats.log 2>&1 || exit $?
echo done
