#!/bin/bash
# small-record leg: repair rounds and section clocks (experiment build), then per-kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
D=gpurun_out/smallprof
mkdir -p $D
timeout -k 10 200 python3 tools/small_once.py libclyscan.so 2 > $D/dbg.log 2>&1 || exit $?
grep -c "repair round" $D/dbg.log; tail -2 $D/dbg.log
timeout -k 10 200 python3 tools/small_once.py libexp_prof.so > $D/prof_small.log 2>&1 || exit $?
tail -3 $D/prof_small.log
timeout -k 10 200 python3 tools/scan_once.py c2 3 libexp_prof.so > $D/prof_c2.log 2>&1 || exit $?
tail -3 $D/prof_c2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o run -- python3 tools/small_once.py libclyscan.so > $D/prof.log 2>&1 || exit $?
find $D/prof -name '*kernel_stats.csv' -exec cat {} \;
