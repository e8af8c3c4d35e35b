#!/bin/bash
# same-box bench lines (C2, C3) of the product and experiment builds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/xpcmp2
mkdir -p $D
for cfg in c2 c3; do
  for lib in "$@"; do
    timeout -k 10 200 python3 tools/scan_once.py $cfg 6 $lib > $D/${cfg}_${lib}.log 2>&1 || exit $?
    tail -1 $D/${cfg}_${lib}.log
  done
done
