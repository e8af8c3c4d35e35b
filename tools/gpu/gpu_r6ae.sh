#!/bin/bash
# round 6: k_emit's tile-wide pass as two half-runs: GPU suite, k_emit A/B against a4a3942
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ae
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for lib in libclyscan.so libexp_a4a3942.so; do
    for c in c3 c5 c2; do
      timeout -k 10 300 python3 tools/scan_once.py $c 4 $lib > $D/${c}_${lib}_$pass.log 2>&1 || exit $?
      tail -1 $D/${c}_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print('$pass $c $lib k_emit %.3f k_scan %.3f all %.3f' % (d['k_emit'], d['k_scan'], d['all']))"
    done
  done
done
