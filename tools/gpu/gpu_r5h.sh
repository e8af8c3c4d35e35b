#!/bin/bash
# GPU suite, then same-box C2 / C3 / small lines of the product and a baseline build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5h
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; tail -3 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/gpu_xpcmp2.sh "$@"
for lib in "$@"; do
  timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_$lib.log 2>&1 || exit $?
  tail -1 $D/small_$lib.log
done
