#!/bin/bash
# same-box k_scan comparison of experiment builds: tools/gpu/gpu_xpcmp.sh CFG LIB...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/xpcmp
mkdir -p $D
cfg=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    timeout -k 10 200 python3 tools/scan_once.py $cfg 12 $lib > $D/${cfg}_${lib}_$rep.log 2>&1 || exit $?
    tail -1 $D/${cfg}_${lib}_$rep.log
  done
done
