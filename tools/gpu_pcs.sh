#!/bin/bash
# PC sampling (host trap) of the C2 scan kernels: which instructions the waves sit on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval 1 --kernel-trace --output-format csv -d gpurun_out/pcs/c2 -o run -- \
  python3 tools/scan_once.py c2 20 > gpurun_out/pcs/c2.log 2>&1
echo "rc=$?"; tail -5 gpurun_out/pcs/c2.log; ls -la gpurun_out/pcs/c2 | head
