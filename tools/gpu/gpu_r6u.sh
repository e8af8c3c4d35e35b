#!/bin/bash
# round 6: why C3 / C5 take a host repair round (cly_dbg_set 2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6u
mkdir -p $D
for c in c3 c5 c4; do
  timeout -k 10 200 python -u tools/repair_probe.py $c > $D/$c.log 2>&1 || exit $?
done
grep -h "repair\|passes" $D/*.log
