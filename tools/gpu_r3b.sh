#!/bin/bash
# GPU tests, then the C4 bench under rocprofv3 kernel stats, then the full C2 bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/c4prof -o run --output-format csv -- python bench.py --config c4 --steps 5 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/r3b/bench_c4.json 2> gpurun_out/r3b/bench_c4.err || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3b/bench_c2.json 2> gpurun_out/r3b/bench_c2.err || exit $?
exit 0
