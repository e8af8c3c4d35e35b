#!/bin/bash
# round 6: skeleton -- segment-register stores vs k_scan checking records itself
# (Kogge-Stone over the lanes + A^(4k) entry registers), 4 GiB
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6q
mkdir -p $D
timeout -k 10 120 ./tools/xp/skel > $D/skel_ks.log 2>&1 || exit $?
cat $D/skel_ks.log
