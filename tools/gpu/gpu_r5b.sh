#!/bin/bash
# skeleton microbench, then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5b
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 120 ./tools/xp/skel > $D/skel.log 2>&1 || exit $?
cat $D/skel.log
timeout -k 10 600 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; tail -25 $D/pytest_gpu.log; exit $rc
