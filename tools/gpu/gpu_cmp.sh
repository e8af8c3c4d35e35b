#!/bin/bash
# same-box C2 kernel stats of the round-3 library and this build, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/cmp
i=0
for lib in libclyscan_r3.so libclyscan.so libclyscan_r3.so libclyscan.so; do
  i=$((i + 1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cmp/${i}_$lib -o run -- \
    python3 tools/scan_once.py c2 10 $lib > gpurun_out/cmp/${i}_$lib.log 2>&1 || exit $?
  tail -1 gpurun_out/cmp/${i}_$lib.log
done
timeout -k 10 400 python -u bench.py > gpurun_out/cmp/bench_c2.json 2> gpurun_out/cmp/bench_c2.err || exit $?
echo done
