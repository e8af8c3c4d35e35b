#!/bin/bash
# round-end artifacts of the final build: GPU suite (slow tests included),
# smoke(), then tools/gpu/gpu_r5prof.sh (same-box round-3 comparison and the default
# bench line, C3/C4 bench lines, kernel stats, SQ and traffic passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/fin
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 300 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -1 $D/smoke.log
bash tools/gpu/gpu_r5prof.sh
