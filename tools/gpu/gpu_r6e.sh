#!/bin/bash
# round 6: write-reduction variants of k_scan's skeleton (8-B entries; segment
# registers at 128-B / 256-B granularity)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6e
mkdir -p $D
timeout -k 10 200 ./tools/xp/skel > $D/skel.log 2>&1 || exit $?
cat $D/skel.log
timeout -k 10 200 ./tools/xp/skel > $D/skel2.log 2>&1 || exit $?
cat $D/skel2.log
