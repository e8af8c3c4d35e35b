#!/bin/bash
# GPU suite, then C4 merge kernel stats of each library in $@ (rocprofv3 --stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mg
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/mg/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/mg/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
i=0
for lib in "$@"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mg/${i}_$lib -o run -- \
    python3 tools/merge_once.py 4 $lib > gpurun_out/mg/${i}_$lib.log 2>&1 || exit $?
  grep "c4 merge" gpurun_out/mg/${i}_$lib.log
done
echo done
