#!/bin/bash
# GPU suite, C3 repair diagnostic, C2/C3 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5d
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; tail -4 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/diag_runs.py c3 4 > $D/diag_c3.log 2>&1 || exit $?
grep -v amdgpu.ids $D/diag_c3.log | tail -12
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-path > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
head -c 1200 $D/bench_c2.json; echo
timeout -k 10 400 python -u bench.py --config c3 --no-host-path --no-cpu-baseline > $D/bench_c3.json 2> $D/bench_c3.err || exit $?
head -c 1200 $D/bench_c3.json; echo
