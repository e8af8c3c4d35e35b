#!/bin/bash
# round 6 diagnosis: streaming microbenchmarks, then k_scan alone with HBM loads vs L2-resident loads
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6a
mkdir -p $D
timeout -k 10 120 ./tools/xp/stream_depth > $D/stream_depth.log 2>&1 || exit $?
cat $D/stream_depth.log
timeout -k 10 120 ./tools/xp/skel > $D/skel.log 2>&1 || exit $?
cat $D/skel.log
for pass in 1 2; do
  for lib in libexp_base.so libexp_l2.so; do
    for cfg in c2 c3; do
      timeout -k 10 300 python3 tools/scan_once.py $cfg 4 $lib > $D/${cfg}_${lib}_$pass.log 2>&1 || exit $?
      echo "$pass $cfg $lib $(tail -1 $D/${cfg}_${lib}_$pass.log | grep -o "'k_scan': [0-9.]*")"
    done
  done
done
