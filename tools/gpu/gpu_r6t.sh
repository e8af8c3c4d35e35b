#!/bin/bash
# round 6: k_refix steps over boundary-less tiles (fewer repair rounds): GPU suite,
# same-box A/B against the r6fin build (95a460b)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6t
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
tail -1 $D/smoke.log
ABDIR=r6t_ab bash tools/gpu/gpu_ab.sh libclyscan.so libexp_95a460b.so
