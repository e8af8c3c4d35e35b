#!/bin/bash
# GPU perf session: parity check (both geometries), bench, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 5 200 python tools/check_lib.py libclyscan_small.so --corpora=8 > gpurun_out/check_small.log 2>&1 || exit $?
timeout -k 5 200 python tools/check_lib.py libclyscan.so --corpora=8 > gpurun_out/check.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 || exit $?
if [[ -n "$PROF" ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
fi
exit 0
