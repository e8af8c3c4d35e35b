#!/bin/bash
# GPU suite, then C2 and C4 kernel stats of the libraries named in $@
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4g
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/r4g/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4g/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
CFG=c2 bash tools/gpu/gpu_xp.sh "$@" || exit $?
CFG=c4 bash tools/gpu/gpu_xp.sh "$@" || exit $?
echo done
