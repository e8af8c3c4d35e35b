#!/bin/bash
# same-box small-record legs of the product and experiment builds, then C2 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/xpsmall
mkdir -p $D
for lib in "$@"; do
  timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_${lib}.log 2>&1 || exit $?
  tail -2 $D/small_${lib}.log
done
for lib in "$@"; do
  timeout -k 10 200 python3 tools/scan_once.py c2 6 $lib > $D/c2_${lib}.log 2>&1 || exit $?
  tail -1 $D/c2_${lib}.log
done
