#!/bin/bash
# section clocks of the small-record leg (prof experiment builds), then a same-box A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/xprof
mkdir -p $D
for lib in libexp_profbase.so libexp_prof.so; do
  timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_$lib.log 2>&1 || exit $?
  grep "xp:" $D/small_$lib.log | tail -2; tail -1 $D/small_$lib.log
  timeout -k 10 300 python3 tools/scan_once.py c3 2 $lib > $D/c3_$lib.log 2>&1 || exit $?
  grep "xp:" $D/c3_$lib.log | tail -1; tail -1 $D/c3_$lib.log
done
bash tools/gpu/gpu_ab.sh "$@"
