#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5f
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; tail -3 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_r5e.sh
