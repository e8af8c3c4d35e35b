#!/bin/bash
# round 6: a second header hop for guesses whose walk leaves the block: repair
# rounds (probe), GPU suite, same-box A/B against d8d2590
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6v
mkdir -p $D
export TMPDIR=/tmp
for c in c3 c5; do
  timeout -k 10 200 python -u tools/repair_probe.py $c > $D/probe_$c.log 2>&1 || exit $?
done
grep -h "repair\|passes" $D/probe_*.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
ABDIR=r6v_ab bash tools/gpu/gpu_ab.sh libclyscan.so libexp_d8d2590.so
