#!/bin/bash
# round 6: k_fin's scan levels from host-built tables A^(CLY_TILE 2^k) (no
# serial square-and-multiply, no bitwise products), tiles loaded four at a
# time: GPU suite, same-box A/B of k_fin against 3d5b41c
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6aj
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -x --timeout 150 --timeout-method thread -m gpu > $D/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $D/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for lib in libclyscan.so libexp_3d5b41c.so; do
    for cfg in c2 c3; do
      timeout -k 10 300 python3 tools/scan_once.py $cfg 4 $lib > $D/${cfg}_${lib}_$pass.log 2>&1 || exit $?
      tail -1 $D/${cfg}_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print('$pass $cfg $lib k_fin %.4f k_emit %.4f all %.3f' % (d['k_fin'], d['k_emit'], d['all']))"
    done
    timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_${lib}_$pass.log 2>&1 || exit $?
    tail -1 $D/small_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.rindex('{'):]); print('$pass small $lib k_fin %.4f k_emit %.4f all %.3f' % (d['k_fin'], d['k_emit'], d['all']))"
  done
done
