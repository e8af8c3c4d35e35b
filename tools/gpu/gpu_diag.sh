#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag_runs.py c3 4 > gpurun_out/diag/c3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/diag/c3.log | tail -25
