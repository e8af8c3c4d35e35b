#!/bin/bash
# SQ instruction counters of k_scan for the full build and the timing-experiment builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/exppmc
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"
for lib in libclyscan.so libclyscan_exp2.so libclyscan_exp3.so libclyscan_exp11.so libclyscan_exp7.so libclyscan_exp4.so; do
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/exppmc/$lib -o run -- python tools/exp_one.py $lib > gpurun_out/exppmc/$lib.log 2>&1 || exit $?
done
exit 0
