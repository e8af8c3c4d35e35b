#!/bin/bash
# One SQ counter pass per library variant (LIBS) over tools/scan_once.py c2:
# per-dispatch instruction counts of k_scan for each build into gpurun_out/pmcv/<lib>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcv
export TMPDIR=/tmp
SET="${SET:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY}"
for lib in ${LIBS:-libclyscan.so}; do
  rm -rf gpurun_out/pmc
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/scan_once.py ${CFG:-c2} 2 $lib > gpurun_out/pmcv/$lib.log 2>&1 || exit $?
  python3 tools/pmc_agg.py ${KERN:-k_scan} > gpurun_out/pmcv/$lib.txt
done
exit 0
