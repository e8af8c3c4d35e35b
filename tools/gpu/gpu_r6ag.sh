#!/bin/bash
# round 6: the small-record file's wrong run-start guesses
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6ag
mkdir -p $D
timeout -k 10 300 python -u tools/guess_probe.py small > $D/guess_small.log 2>&1 || exit $?
grep -v "amdgpu.ids" $D/guess_small.log | tail -16 | cut -c1-330
