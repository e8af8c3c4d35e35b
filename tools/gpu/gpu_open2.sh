#!/bin/bash
# index-load probe: C2 files in /dev/shm; the product library opened twice in a
# fresh process, with SDMA copies (default) and with blit-kernel copies
# (HSA_ENABLE_SDMA=0), twice each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/open
D=$(mktemp -d /dev/shm/clyprobe_XXXX)
trap 'rm -rf "$D"' EXIT
timeout -k 10 300 python -u tools/open_probe.py gen "$D" c2 || exit $?
for k in 1 2; do
  timeout -k 10 120 python -u tools/open_probe.py open "$D" libclyscan.so 2>&1 | tee -a gpurun_out/open/probe2.log || exit $?
  HSA_ENABLE_SDMA=0 timeout -k 10 120 python -u tools/open_probe.py open "$D" libclyscan.so 2>&1 | sed 's/^/nosdma /' | tee -a gpurun_out/open/probe2.log || exit $?
done
echo done
