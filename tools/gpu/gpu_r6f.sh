#!/bin/bash
# round 6: stores behind a counted wait vs a vmcnt(0) wait (tools/xp/waitcnt.hip)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r6f
mkdir -p $D
timeout -k 10 200 ./tools/xp/waitcnt > $D/waitcnt.log 2>&1 || exit $?
cat $D/waitcnt.log
