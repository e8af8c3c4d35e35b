#!/bin/bash
# GPU parity tests (and optional bench), each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TLIM:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYARGS} > gpurun_out/pytest_gpu.log 2>&1 || exit $?
if [[ -n "$BENCH" ]]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
fi
exit 0
