#!/bin/bash
# round 6: GPU suite of this build, then a same-box A/B against the previous commit's library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6g
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_ab.sh libclyscan.so libexp_8137098.so
