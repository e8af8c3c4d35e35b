#!/bin/bash
# index-load probe: C2 files in /dev/shm, then each library in $@ opened twice in a fresh process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/open
D=$(mktemp -d /dev/shm/clyprobe_XXXX)
trap 'rm -rf "$D"' EXIT
timeout -k 10 300 python -u tools/open_probe.py gen "$D" c2 || exit $?
for lib in "$@"; do
  timeout -k 10 120 python -u tools/open_probe.py open "$D" $lib 2>&1 | tee -a gpurun_out/open/probe.log || exit $?
done
echo done
