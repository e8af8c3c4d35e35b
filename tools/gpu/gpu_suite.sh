#!/bin/bash
# GPU suite (slow tests included) and the default bench line of this build; $1 = output dir name
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${1:-suite}
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $D/bench_c2.json 2> $D/bench_c2.err || exit $?
cat $D/bench_c2.json
