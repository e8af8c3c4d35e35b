#!/bin/bash
# round 6: wall-clock A/B of the second-hop guess check (C3, C5, C2) against d8d2590
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6w
mkdir -p $D
for c in c3 c5 c2; do
  timeout -k 10 300 python -u tools/wall_ab.py $c libclyscan.so libexp_d8d2590.so > $D/wall_$c.log 2>&1 || exit $?
done
grep -h "wall" $D/wall_*.log
