#!/bin/bash
# full GPU suite, the default bench (C2 with host path and index load), C4 and
# C3 benches, the C4 kernel stats, experiment libs' C2 kernel stats ($@)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4e/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/r4e/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r4e/bench_c2.json 2> gpurun_out/r4e/bench_c2.err || exit $?
CFG=c2 bash tools/gpu/gpu_xp.sh libclyscan.so "$@" || exit $?
timeout -k 10 400 python -u bench.py --config c4 --no-host-path --no-cpu-baseline > gpurun_out/r4e/bench_c4.json 2> gpurun_out/r4e/bench_c4.err || exit $?
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4e/c4_stats -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-host-path --no-cpu-baseline > gpurun_out/r4e/c4_stats.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --config c3 --no-host-path --no-cpu-baseline > gpurun_out/r4e/bench_c3.json 2> gpurun_out/r4e/bench_c3.err || exit $?
echo done
CFG=c3 bash tools/gpu/gpu_xp.sh libclyscan.so libclyscan_head.so || exit $?
echo done2
