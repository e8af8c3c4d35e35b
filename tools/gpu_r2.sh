#!/bin/bash
# round-2 GPU check: parity tests, bench (C2), per-phase cycle profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TLIM:-500} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYARGS} > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
if [[ -n "$PHASE" ]]; then
  timeout -k 10 200 python tools/phase_prof.py c2 > gpurun_out/phase.log 2>&1 || exit $?
fi
exit 0
