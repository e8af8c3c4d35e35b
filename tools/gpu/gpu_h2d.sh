#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/h2d
mkdir -p $D
export CLY_XP_TIMES=1
for m in 0; do
  timeout -k 10 200 python3 tools/h2d_ab.py $m > $D/m$m.log 2>&1 || exit $?
  grep "xp open\|mode" $D/m$m.log
done
