#!/bin/bash
# round 6: where C3's k_scan time goes (section clocks, general-pass counters)
# on C3, C2 and the small-record file
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6p
mkdir -p $D
export TMPDIR=/tmp
for lib in libexp_prof.so libexp_cnt.so libclyscan.so; do
  for c in c3 c2; do
    timeout -k 10 200 python -u tools/scan_once.py $c 3 $lib > $D/${c}_$lib.log 2>&1 || exit $?
  done
  timeout -k 10 200 python -u tools/small_once.py $lib > $D/small_$lib.log 2>&1 || exit $?
done
grep -h "xp:\|k_scan" $D/*.log | cut -c1-400
echo done
