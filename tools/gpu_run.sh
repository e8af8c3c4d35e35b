#!/bin/bash
# GPU session: fixture/corpus check of both geometries, parity tests, smoke,
# short bench.  Each GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGES="${1:-check,pytest,smoke,bench}"
run() { echo "== $1" >> gpurun_out/steps.log; }
if [[ $STAGES == *check* ]]; then
  run check
  timeout -k 10 300 python tools/check_lib.py libclyscan_small.so --corpora=12 > gpurun_out/check_small.log 2>&1 || exit $?
  timeout -k 10 300 python tools/check_lib.py libclyscan.so --corpora=12 > gpurun_out/check.log 2>&1 || exit $?
fi
if [[ $STAGES == *pytest* ]]; then
  run pytest
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
fi
if [[ $STAGES == *smoke* ]]; then
  run smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
fi
if [[ $STAGES == *bench* ]]; then
  run bench
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
fi
exit 0
