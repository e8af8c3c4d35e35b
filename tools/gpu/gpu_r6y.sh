#!/bin/bash
# round 6: second header hop in an out-of-line guess_entry (only without a confirmed start):
# block: repair rounds (probe), GPU suite, wall-clock A/B against d8d2590
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6y
mkdir -p $D
export TMPDIR=/tmp
for c in c3 c5; do
  timeout -k 10 200 python -u tools/repair_probe.py $c > $D/probe_$c.log 2>&1 || exit $?
done
grep -h "repair\|passes" $D/probe_*.log | cut -c1-200
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for c in c3 c5 c2; do
  timeout -k 10 300 python -u tools/wall_ab.py $c libclyscan.so libexp_d8d2590.so > $D/wall_$c.log 2>&1 || exit $?
done
grep -h "wall" $D/wall_*.log
