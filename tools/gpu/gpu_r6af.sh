#!/bin/bash
# round 6: the small-record file's link phase (repair rounds, kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6af
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/small_once.py libclyscan.so 2 > $D/small_dbg.log 2>&1 || exit $?
grep -v amdgpu.ids $D/small_dbg.log | tail -5 | cut -c1-300
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/small_stats -o run -- python3 tools/small_once.py libclyscan.so > $D/small_stats.log 2>&1 || exit $?
echo done
