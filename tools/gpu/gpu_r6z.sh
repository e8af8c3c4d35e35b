#!/bin/bash
# round 6: C2 / C5 wall-clock A/B of the inline second-hop guess check, both orders
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6z
mkdir -p $D
for c in c2 c5; do
  timeout -k 10 300 python -u tools/wall_ab.py $c libexp_d8d2590.so libclyscan.so > $D/wall_${c}_ba.log 2>&1 || exit $?
  timeout -k 10 300 python -u tools/wall_ab.py $c libclyscan.so libexp_d8d2590.so > $D/wall_${c}_ab.log 2>&1 || exit $?
done
grep -h "wall" $D/wall_*.log
