#!/bin/bash
# round 6: which run-start guesses C3 / C5 still get wrong
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6aa
mkdir -p $D
for c in c3 c5; do
  timeout -k 10 300 python -u tools/guess_probe.py $c > $D/guess_$c.log 2>&1 || exit $?
done
grep -hv "amdgpu.ids" $D/guess_*.log | cut -c1-330
