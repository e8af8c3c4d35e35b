#!/bin/bash
# round 6: k_emit loads the next tile's segment registers while it works on
# the current one: GPU suite, same-box A/B against eb8ff66 (k_emit by markers)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6al
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for lib in libclyscan.so libexp_eb8ff66.so; do
    for cfg in c2 c3 c5; do
      timeout -k 10 300 python3 tools/scan_once.py $cfg 4 $lib > $D/${cfg}_${lib}_$pass.log 2>&1 || exit $?
      tail -1 $D/${cfg}_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print('$pass $cfg $lib k_emit %.4f k_scan %.3f all %.3f' % (d['k_emit'], d['k_scan'], d['all']))"
    done
    timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_${lib}_$pass.log 2>&1 || exit $?
    tail -1 $D/small_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.rindex('{'):]); print('$pass small $lib k_emit %.4f k_scan %.3f all %.3f' % (d['k_emit'], d['k_scan'], d['all']))"
  done
done
