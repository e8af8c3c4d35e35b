#!/bin/bash
# Quick GPU parity check of both geometries (fixtures + random corpora, normal and
# forced wrong-guess paths), then an optional bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/check_lib.py libclyscan_small.so --corpora=${NCORP:-4} > gpurun_out/check_small.log 2>&1 || exit $?
timeout -k 10 120 python tools/check_lib.py libclyscan.so --corpora=${NCORP:-4} > gpurun_out/check.log 2>&1 || exit $?
timeout -k 10 120 python tools/check_lib.py libclyscan_small.so --corpora=4 --force-redo > gpurun_out/check_small_redo.log 2>&1 || exit $?
timeout -k 10 120 python tools/check_lib.py libclyscan.so --corpora=4 --force-redo > gpurun_out/check_redo.log 2>&1 || exit $?
if [[ -n "$BENCH" ]]; then
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-path ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
fi
exit 0
