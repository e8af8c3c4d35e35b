#!/bin/bash
# GPU suite (with the slow tests), then the small-record leg and C2 / C3 kernel lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r5g
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; tail -5 $D/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/small_once.py libclyscan.so > $D/small.log 2>&1 || exit $?
tail -1 $D/small.log
for cfg in c2 c3; do
  timeout -k 10 300 python3 tools/scan_once.py $cfg 4 libclyscan.so > $D/$cfg.log 2>&1 || exit $?
  tail -1 $D/$cfg.log
done
