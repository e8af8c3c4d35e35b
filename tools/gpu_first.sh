#!/bin/bash
# First GPU contact: debug-build fixture scan, then parity tests, smoke, short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== go: $(go version 2>&1 | head -1)" > gpurun_out/env.txt
nproc >> gpurun_out/env.txt
rocm-smi --showproductname >> gpurun_out/env.txt 2>&1 || true
timeout -k 10 240 python tools/debug_scan.py libclyscan_small_dbg.so > gpurun_out/dbg_small.log 2>&1 \
 && timeout -k 10 240 python tools/debug_scan.py libclyscan_dbg.so > gpurun_out/dbg.log 2>&1 \
 && timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "not slow" > gpurun_out/pytest_gpu.log 2>&1
