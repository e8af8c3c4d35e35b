#!/bin/bash
# k_scan alone (SCAN_ONLY builds): stores kept vs removed, C2 and C3; then the open probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/xpns
mkdir -p $D
for pass in 1 2; do
  for lib in libexp_base.so libexp_nostore.so; do
    for cfg in c2 c3; do
      timeout -k 10 300 python3 tools/scan_once.py $cfg 4 $lib > $D/${cfg}_${lib}_$pass.log 2>&1 || exit $?
      echo "$pass $cfg $lib $(tail -1 $D/${cfg}_${lib}_$pass.log | grep -o "'k_scan': [0-9.]*")"
    done
  done
done
