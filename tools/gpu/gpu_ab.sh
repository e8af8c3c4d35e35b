#!/bin/bash
# same-box A/B: C2, C3 and small-record kernel lines of each build, two passes (A B A B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/${ABDIR:-ab}
mkdir -p $D
for pass in 1 2; do
  for lib in "$@"; do
    for cfg in c2 c3; do
      timeout -k 10 300 python3 tools/scan_once.py $cfg 4 $lib > $D/${cfg}_${lib}_$pass.log 2>&1 || exit $?
      tail -1 $D/${cfg}_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.index('{'):]); print('$pass $cfg $lib k_scan %.3f all %.3f' % (d['k_scan'], d['all']))"
    done
    timeout -k 10 200 python3 tools/small_once.py $lib > $D/small_${lib}_$pass.log 2>&1 || exit $?
    tail -1 $D/small_${lib}_$pass.log | python3 -c "import sys,ast; l=sys.stdin.read(); d=ast.literal_eval(l[l.rindex('{'):]); print('$pass small $lib k_scan %.3f all %.3f' % (d['k_scan'], d['all']))"
  done
done
