#!/bin/bash
# round 6: general-pass output owners from a wave sum of first-record bits
# (no per-round search over the lanes): GPU suite, same-box A/B against 355bc01
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ai
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ABDIR=r6ai_ab bash tools/gpu/gpu_ab.sh libclyscan.so libexp_355bc01.so
