#!/bin/bash
# One GPU session: parity check (both geometries), pytest -m gpu, smoke, bench,
# rocprofv3 kernel stats.  Each GPU step has its own time limit; first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python tools/check_lib.py libclyscan_small.so --corpora=8 > gpurun_out/check_small.log 2>&1 || exit $?
timeout -k 10 200 python tools/check_lib.py libclyscan.so --corpora=8 > gpurun_out/check.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
if [[ -n "$PROF" ]]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-path > gpurun_out/prof.log 2>&1 || exit $?
fi
exit 0
