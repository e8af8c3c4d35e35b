#!/bin/bash
# full GPU suite, the default bench (C2 with host path and index load), experiment libs' C2 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4e/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4e/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r4e/bench_c2.json 2> gpurun_out/r4e/bench_c2.err || exit $?
CFG=c2 bash tools/gpu_xp.sh "$@"
